import json, sys
L = json.load(open(sys.argv[1]))
order = []
for l in L:
    if l['root'] not in order: order.append(l['root'])
n = int(sys.argv[2]) if len(sys.argv) > 2 else 6
tot = {}
for r in order:
    ls = [l for l in L if l['root'] == r]
    tot[r] = ls[-1]['cum_ms']
worst = sorted(order, key=lambda r: -tot[r])[:3]
for r in order[:n] + worst:
    ls = [l for l in L if l['root'] == r]
    print('root', r, 'total %.3f' % ls[-1]['cum_ms'])
    for l in ls:
        print('  L%d %s fin=%d fout=%d mf=%d unv=%d scan=%d claims=%d k=%.3f cum=%.3f' % (l['level'], 'TD' if l['direction'] == 1 else 'BU', l['frontier_in'], l['frontier_out'], l['mf_in'], l['unvisited_in'], l['scanned'], l.get('claims', 0), l['kernel_ms'], l['cum_ms']))
