"""Summarise tools/pmc_busy.sh's counter passes per kernel (dev tool).

Per kernel (averaged over its dispatches):
  mfma_busy  = SQ_VALU_MFMA_BUSY_CYCLES / (kernel cycles x 1024 SIMDs), the
               matrix pipe's busy fraction (the counter sums MFMA busy cycles,
               e.g. 16 per v_mfma_f32_16x16x32_f16, over the chip);
  valu_busy  = 4 x SQ_ACTIVE_INST_VALU / (kernel cycles x 1024 SIMDs) (the
               SQ_ACTIVE_* counters are in quad-cycles);
  kernel cycles = GRBM_GUI_ACTIVE / 8 (rocprofv3 sums it over the 8 XCDs);
  wait_any / wait_inst / active = shares of SQ_WAVE_CYCLES (parked on
               s_waitcnt or a barrier / issue-stalled / issuing);
  insts per wave-instruction mix: SQ_INSTS_{VALU,MFMA,LDS,SALU,VMEM}.
Calibration (din_head read valu_busy 1.02): the raw formulas
above are divided by what the pure loops of tools/calib/calib.hip read under
the same counters (DIR/cal{1,2}): mfma_loop (back-to-back MFMAs, matrix pipe
saturated) and valu_loop (independent v_fma_f32, 8 waves per SIMD, VALU issue
saturated).  SQ_ACTIVE_INST_VALU counts each wave's VALU issue time, and
waves on one SIMD overlap there, so the raw VALU formula of a saturated SIMD
reads about 2, not 1.  Both raw and calibrated values are written.
usage: pmc_busy.py DIR  (DIR/{scr,din,cal}{1,2}/.../run_counter_collection.csv)
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

SIMDS = 256 * 4
KEEP = ("ip_screen", "ip_scan", "ip_select", "ip_refine", "din_att_h", "din_wh", "din_mlp1", "din_mlp2", "din_head", "tt_user",
        "din_att_stats", "din_att_wh", "din_att_tm", "din_tm_plan")


def load(path):
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        per = defaultdict(lambda: defaultdict(float))
        names = {}
        for r in csv.DictReader(open(f)):
            d = int(r["Dispatch_Id"])
            names[d] = r["Kernel_Name"].split("(")[0].replace("void ", "")
            per[d][r["Counter_Name"]] += float(r["Counter_Value"])
        for d, cs in per.items():
            for c, v in cs.items():
                vals[names[d]][c].append(v)
    return vals


def raw_busy(c):
    cyc = c.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
    if not cyc:
        return None, None, cyc
    return (c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (cyc * SIMDS),
            4.0 * c.get("SQ_ACTIVE_INST_VALU", 0.0) / (cyc * SIMDS), cyc)


def merged(root, grp):
    m = defaultdict(dict)
    for i in (1, 2):
        for k, cs in load(os.path.join(root, f"{grp}{i}")).items():
            for c, v in cs.items():
                m[k][c] = sum(v) / len(v)
    return m


def main():
    root = sys.argv[1]
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench

    cal = merged(root, "cal")
    cm = [raw_busy(c)[0] for k, c in cal.items() if "mfma_loop" in k]
    cv = [raw_busy(c)[1] for k, c in cal.items() if "valu_loop" in k]
    cal_mfma = cm[0] if cm and cm[0] else 1.0
    cal_valu = cv[0] if cv and cv[0] else 1.0
    out = {"sources": bench.source_digest(),
           "calibration": {"mfma_loop_raw_mfma_busy": cal_mfma, "valu_loop_raw_valu_busy": cal_valu,
                           "note": "mfma_busy / valu_busy below = raw formula / these pure-loop readings"},
           "kernels": {}}
    for grp in ("scr", "din", "cal"):
        for k, c in merged(root, grp).items():
            if grp != "cal" and not any(s in k for s in KEEP):
                continue
            mb, vb, cyc = raw_busy(c)
            wc = c.get("SQ_WAVE_CYCLES", 0.0)
            r = {"kernel_cycles": round(cyc)}
            if cyc:
                r["mfma_busy"] = round(mb / cal_mfma, 4)
                r["valu_busy"] = round(vb / cal_valu, 4)
                r["mfma_busy_raw"] = round(mb, 4)
                r["valu_busy_raw"] = round(vb, 4)
            if wc:
                for n, key in (("wait_any", "SQ_WAIT_ANY"), ("wait_inst", "SQ_WAIT_INST_ANY"),
                               ("active", "SQ_ACTIVE_INST_ANY")):
                    r[n] = round(c.get(key, 0.0) / wc, 4)
            for key in ("SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_VMEM",
                        "SQ_LDS_BANK_CONFLICT", "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS"):
                if key in c:
                    r[key] = c[key]
            out["kernels"][k] = r
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
