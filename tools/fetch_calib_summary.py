"""Join tools/fetch_calib's known bytes with its rocprofv3 FETCH_SIZE / WRITE_SIZE passes.

  python tools/fetch_calib_summary.py <dir with calib.json, pmc_fetch/, pmc_write/> <out.json>

For every calibration kernel: the counter's bytes per launch (KiB x 1024, mean over its launches), the
bytes the kernel is known to move (distinct 64-B lines x 64, or the streamed bytes) and their ratio
`factor` = known / counted: multiply a counter reading of that access class by it to get the bytes moved."""
import csv
import json
import os
import statistics as S
import sys


def per_kernel(path):
    out = {}
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].replace("void ", "").split("(")[0].strip()
        out.setdefault(name, []).append(float(r["Counter_Value"]) * 1024.0)
    return out


def main():
    d, dst = sys.argv[1], sys.argv[2]
    known = json.load(open(os.path.join(d, "calib.json")))
    fetch = per_kernel(os.path.join(d, "pmc_fetch", "run_counter_collection.csv"))
    write = per_kernel(os.path.join(d, "pmc_write", "run_counter_collection.csv"))
    res = {"array_bytes": known["array_bytes"], "kernels": {},
           "note": "factor = known bytes / counter bytes (KiB x 1024); apply to a counter reading of the same "
                   "access class.  Scattered kernels touch distinct 64-B lines of an 8 GiB array (32x the "
                   "Infinity Cache)"}
    for k, kn in known["kernels"].items():
        e = {"known_read_B": kn["known_read_bytes_per_launch"], "known_write_B": kn["known_write_bytes_per_launch"],
             "ms": kn["ms"]}
        if k in fetch:
            e["fetch_B"] = S.mean(fetch[k])
            if e["known_read_B"]:
                e["fetch_factor"] = round(e["known_read_B"] / e["fetch_B"], 4) if e["fetch_B"] else None
        if k in write:
            e["write_B"] = S.mean(write[k])
            if e["known_write_B"]:
                e["write_factor"] = round(e["known_write_B"] / e["write_B"], 4) if e["write_B"] else None
        res["kernels"][k] = e
    json.dump(res, open(dst, "w"), indent=1)
    for k, e in res["kernels"].items():
        print(k, {x: e.get(x) for x in ("fetch_factor", "write_factor", "ms")})


if __name__ == "__main__":
    main()
