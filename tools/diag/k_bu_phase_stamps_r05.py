"""Round-5 form of k_bu_phase_stamps.patch (the patch is against the pre-split kernels_bfs.hip): adds the
s_memtime phase stamps (compaction / A1 / A2 / B) to k_bu in a COPY of the sources and reports the per-level cycle
sums in place of the level counters scanned / claims / stage2 / walked.   usage:
    python tools/diag/k_bu_phase_stamps_r05.py <copy>/bfs-with-mapreduce_amd/csrc/kernels_pull.hip
then build that copy's libbfsx.so and run  BFSX_LIB=<copy>/.../libbfsx.so python bench.py --levels-json ...
Never applied to the product tree."""
import sys

p = sys.argv[1]
s = open(p).read()


def rep(old, new):
    global s
    assert s.count(old) == 1, (old[:60], s.count(old))
    s = s.replace(old, new)


rep('''    const int64_t wstride = (int64_t)gridDim.x * kWaves * 64;
    for (int64_t w0 = ((int64_t)blockIdx.x * kWaves + wave) * 64; w0 < nwords; w0 += wstride) {''',
    '''    uint32_t tph[4] = {0, 0, 0, 0}; // DIAG: cycles in compaction/group, A1, A2, B
    u64 tprev = __builtin_amdgcn_s_memtime();
    auto stamp = [&](int ph) { const u64 t = __builtin_amdgcn_s_memtime(); tph[ph] += (uint32_t)(t - tprev); tprev = t; };
    const int64_t wstride = (int64_t)gridDim.x * kWaves * 64;
    for (int64_t w0 = ((int64_t)blockIdx.x * kWaves + wave) * 64; w0 < nwords; w0 += wstride) {''')
rep('''            uint32_t xn[kU]; // kPipe: top1 of the next round's candidates, in flight
            if (kPipe) {''', '''            uint32_t xn[kU]; // kPipe: top1 of the next round's candidates, in flight
            stamp(0);
            if (kPipe) {''')
rep('''                for (int k = 0; k < kU; k++) fbm |= ((pw[k] >> ((x[k] & ~fmask) & 31u)) & 1u) << k;
''', '''                for (int k = 0; k < kU; k++) fbm |= ((pw[k] >> ((x[k] & ~fmask) & 31u)) & 1u) << k;
                stamp(1);
''')
rep('''                        pbm |= (fbit(r[k].x) | (fbit(r[k].y) << 1) | (fbit(r[k].z) << 2)) << (3 * k);
                }
''', '''                        pbm |= (fbit(r[k].x) | (fbit(r[k].y) << 1) | (fbit(r[k].z) << 2)) << (3 * k);
                }
                stamp(2);
''')
rep('''                __builtin_amdgcn_wave_barrier();
                // B: rows longer than 4''', '''                __builtin_amdgcn_wave_barrier();
                stamp(1);
                // B: rows longer than 4''')
rep('''                nmiss -= nb;
                __builtin_amdgcn_wave_barrier();
''', '''                nmiss -= nb;
                __builtin_amdgcn_wave_barrier();
                stamp(3);
''')
rep('''    shard_add(cn, acc_nf, acc_mf, acc_sc, acc_rows, acc_mu, 0, acc_s2, acc_wk, acc_nh);
    publish_if_last(cn, pub, seq);
}

#define BFSX_K_BU_PARAMS''', '''    stamp(0);
    (void)acc_sc; (void)acc_rows; (void)acc_s2; (void)acc_wk;
    shard_add(cn, acc_nf, acc_mf, tph[0], tph[1], acc_mu, 0, tph[2], tph[3], acc_nh);
    publish_if_last(cn, pub, seq);
}

#define BFSX_K_BU_PARAMS''')
open(p, "w").write(s)
