"""Summarise tools/lib_ab.sh: per GEMM shape / attention case the best of the two runs per build,
and the bench values."""
import json
import os
import re
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/lib_ab"


def runs(kind):
    return [(v, r, f"{d}/{kind}_{v}_{r}.log") for v in ("base", "alt") for r in (1, 2)
            if os.path.exists(f"{d}/{kind}_{v}_{r}.log")]


best = {}
for v, r, path in runs("gemm"):
    for line in open(path):
        m = re.match(r"(\w+)\s+(\w+)\s+(\w+)\s+M=.*?\s([\d.]+) ms", line)
        if m:
            best.setdefault(m.group(1, 2, 3), {}).setdefault(v, []).append(float(m.group(4)))
if best:
    tb = ta = 0.0
    for k, x in best.items():
        b, a = min(x["base"]), min(x["alt"])
        tb += b; ta += a
        print(f"{' '.join(k):18s} base {b * 1e3:8.1f} us  alt {a * 1e3:8.1f} us  {b / a:6.3f}x")
    print(f"gemm sum: base {tb * 1e3:.1f} us, alt {ta * 1e3:.1f} us ({tb / ta:.3f}x)")
att = {}
for v, r, path in runs("attn"):
    for line in open(path):
        m = re.match(r"(.*?):\s+fwd\s+([\d.]+) us.*bwd\s+([\d.]+) us", line)
        if m:
            att.setdefault(m.group(1).strip(), {}).setdefault(v, []).append((float(m.group(2)), float(m.group(3))))
for k, x in att.items():
    bf, bb = min(t[0] for t in x["base"]), min(t[1] for t in x["base"])
    af, ab = min(t[0] for t in x["alt"]), min(t[1] for t in x["alt"])
    print(f"{k:34s} fwd base {bf:7.1f} alt {af:7.1f} ({bf / af:5.3f}x)  bwd base {bb:7.1f} alt {ab:7.1f} ({bb / ab:5.3f}x)")
for v in ("base", "alt"):
    vals = []
    for vv, r, path in runs("bench"):
        if vv == v:
            lines = [l for l in open(path) if l.startswith("{")]
            vals.append(json.loads(lines[-1])["value"] if lines else None)
    if vals:
        print(v, "bench", vals)
