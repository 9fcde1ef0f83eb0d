"""Summarise tools/lib_ab.sh: per GEMM shape the best of two runs per build, and the bench values."""
import json
import re
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/lib_ab"
best = {}
for v in ("base", "alt"):
    for r in (1, 2):
        for line in open(f"{d}/gemm_{v}_{r}.log"):
            m = re.match(r"(\w+)\s+(\w+)\s+(\w+)\s+M=.*?\s([\d.]+) ms", line)
            if m:
                k = m.group(1, 2, 3)
                best.setdefault(k, {}).setdefault(v, []).append(float(m.group(4)))
tb = ta = 0.0
for k, x in best.items():
    b, a = min(x["base"]), min(x["alt"])
    tb += b; ta += a
    print(f"{' '.join(k):18s} base {b * 1e3:8.1f} us  alt {a * 1e3:8.1f} us  {b / a:6.3f}x")
print(f"sum: base {tb * 1e3:.1f} us, alt {ta * 1e3:.1f} us ({tb / ta:.3f}x)")
for v in ("base", "alt"):
    vals = []
    for r in (1, 2):
        lines = [l for l in open(f"{d}/bench_{v}_{r}.log") if l.startswith("{")]
        vals.append(json.loads(lines[-1])["value"])
    print(v, "bench", vals)
