"""Fold tools/pmc_mfma.sh output into profiles/<tag>_mfma.json: per kernel (summed over its
dispatches) MFMA FLOPs (MOPS x 512), MFMA utilisation = SQ_VALU_MFMA_BUSY_CYCLES / (GPU cycles x
1024 SIMDs) with GPU cycles = GRBM_GUI_ACTIVE / 8 (rocprofv3 sums the 8 XCDs, MI355X_MICROARCH.md
'DVFS give-back'), VALU instructions per MFMA, and the wait share SQ_WAIT_ANY / SQ_WAVE_CYCLES.

usage: python tools/pmc_mfma_summary.py gpurun_out/prof_<tag> <tag>
"""
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import ROOT, short_name  # noqa: E402


def main(src, tag):
    path = sorted(glob.glob(os.path.join(src, "mfma", "**", "*counter_collection.csv"), recursive=True))[0]
    per = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            k = short_name(row["Kernel_Name"])
            d = per.setdefault(k, {"dispatches": set()})
            d["dispatches"].add(row["Dispatch_Id"])
            d[row["Counter_Name"]] = d.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
    out = {}
    for k, d in per.items():
        n = len(d["dispatches"])
        cyc = d.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
        mfma = d.get("SQ_INSTS_MFMA", 0.0)
        flops = 512.0 * (d.get("SQ_INSTS_VALU_MFMA_MOPS_F32", 0.0) + d.get("SQ_INSTS_VALU_MFMA_MOPS_BF16", 0.0))
        out[k] = {"dispatches": n, "mfma_flops_per_dispatch": flops / max(n, 1),
                  "mfma_util": d.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / max(cyc * 1024.0, 1.0),
                  "valu_per_mfma": d.get("SQ_INSTS_VALU", 0.0) / max(mfma, 1.0),
                  "wait_any_frac": d.get("SQ_WAIT_ANY", 0.0) / max(d.get("SQ_WAVE_CYCLES", 0.0), 1.0),
                  "gpu_cycles_per_dispatch": cyc / max(n, 1),
                  "raw": {c: v for c, v in d.items() if c != "dispatches"}}
    prof = os.path.join(ROOT, "profiles")
    with open(os.path.join(prof, f"{tag}_mfma.json"), "w") as f:
        json.dump({"tag": tag, "source": "rocprofv3 --pmc (one pass) over python3 bench.py --steps 2 --warmup 1 "
                   "--no-cpu-baseline " + os.environ.get("BENCH_ARGS", ""), "kernels": out}, f, indent=1)
    top = sorted(out.items(), key=lambda kv: -kv[1]["mfma_flops_per_dispatch"] * kv[1]["dispatches"])[:8]
    for k, v in top:
        print(f"{k}: util {v['mfma_util']:.3f} valu/mfma {v['valu_per_mfma']:.2f} wait {v['wait_any_frac']:.2f}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
