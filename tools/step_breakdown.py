"""Per-step kernel time by category from a committed rocprofv3 --stats summary
(profiles/<tag>_kernel_stats.csv): steps = adamw_kernel launches.  python tools/step_breakdown.py <csv>"""
import csv
import sys

CATS = [("gemm", ("gemm", "splitk_reduce", "colsum", "reduce_partials")), ("attention", ("attn_",)),
        ("layernorm", ("ln_", "layernorm")), ("operand split", ("split3",)), ("adamw", ("adamw",))]
rows = list(csv.DictReader(open(sys.argv[1])))
steps = sum(int(r["Calls"]) for r in rows if "adamw_kernel" in r["Name"]) or 1
tot = {}
for r in rows:
    cat = next((c for c, keys in CATS if any(k in r["Name"] for k in keys)), "other")
    tot[cat] = tot.get(cat, 0.0) + float(r["TotalDurationNs"]) / 1e6 / steps
print(f"{sys.argv[1]}: {steps} steps; ms per step: " + ", ".join(f"{k} {v:.1f}" for k, v in
                                                              sorted(tot.items(), key=lambda kv: -kv[1]))
      + f"; total {sum(tot.values()):.1f}")
