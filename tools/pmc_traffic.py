"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into
profiles/<round>_traffic.json (HBM-side bytes per launch).

Corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE / WRITE_SIZE are
reported in KiB-like units of 1024 B; on gfx950 FETCH_SIZE counts exactly
half of the bytes of wide coalesced reads, so it is doubled; WRITE_SIZE is
taken as is.  Both include Infinity-Cache hits (memory-side L2 requests).

usage: pmc_traffic.py RECALL_FETCH RECALL_WRITE DIN_FETCH DIN_WRITE OUT
  RECALL_*: passes over `bench.py --steps 1 --warmup 0 --no-din --no-cpu-baseline`
  DIN_*:    passes over `tools/din_prof.py 2` (two DIN config-3 passes); the
            "din_pass" entry sums every launch dispatched by the LAST
            nrk_din_forward_segments call (after the previous pass's
            din_head_kernel, up to and including the last one).
"""
import csv
import json
import sys
from collections import defaultdict


def rows(path, counter):
    out = []
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            out.append((int(r["Dispatch_Id"]), r["Kernel_Name"].split("(")[0].replace("void ", ""),
                        float(r["Counter_Value"]) * 1024.0))
    out.sort()
    return out


def per_kernel(fetch, write):
    f, w = defaultdict(list), defaultdict(list)
    for _, k, v in rows(fetch, "FETCH_SIZE"):
        f[k].append(2.0 * v)
    for _, k, v in rows(write, "WRITE_SIZE"):
        w[k].append(v)
    res = {}
    for k in sorted(set(f) | set(w)):
        fb = sum(f[k]) / len(f[k]) if f[k] else 0.0
        wb = sum(w[k]) / len(w[k]) if w[k] else 0.0
        res[k] = {"launches": max(len(f[k]), len(w[k])), "fetch_bytes_per_launch": fb,
                  "write_bytes_per_launch": wb, "traffic_bytes_per_launch": fb + wb}
    return res


def din_pass(fetch, write):
    """Bytes of the last DIN pass: every dispatch from the last
    din_att_h_kernel's pass start (the first dispatch after the previous
    pass's din_head_kernel) to the end."""
    out = {}
    for name, path, counter, scale in (("fetch", fetch, "FETCH_SIZE", 2.0), ("write", write, "WRITE_SIZE", 1.0)):
        rs = rows(path, counter)
        heads = [i for i, (_, k, _) in enumerate(rs) if "din_head_kernel" in k]
        start = heads[-2] + 1 if len(heads) >= 2 else 0
        end = heads[-1] + 1
        out[name] = sum(scale * v for _, _, v in rs[start:end])
        out[name + "_launches"] = end - start
        out["kernels"] = sorted({k for _, k, _ in rs[start:end]})
    return {"fetch_bytes": out["fetch"], "write_bytes": out["write"],
            "traffic_bytes": out["fetch"] + out["write"], "launches": out["fetch_launches"],
            "kernels": out["kernels"]}


def main(rf, rw, df, dw, out):
    import os

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench

    json.dump({"sources": bench.source_digest(), "source": [rf, rw, df, dw],
               "correction": "FETCH_SIZE x1024 x2, WRITE_SIZE x1024",
               "kernels": per_kernel(rf, rw), "din_kernels": per_kernel(df, dw),
               "din_pass": din_pass(df, dw)}, open(out, "w"), indent=1)


if __name__ == "__main__":
    main(*sys.argv[1:6])
