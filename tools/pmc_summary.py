"""Fold the rocprofv3 outputs of tools/profile.sh into committed summaries under profiles/:

  profiles/<tag>_kernel_stats.csv   per-kernel time summary (rocprofv3 --kernel-trace --stats)
  profiles/<tag>_hbm_traffic.json   per-kernel HBM bytes per dispatch from the two PMC passes:
                                    FETCH_SIZE x 2 (gfx950 reports half of a wide streaming read,
                                    MI355X_MICROARCH.md "HBM") + WRITE_SIZE, both in KB -> bytes
  profiles/<tag>_bench_trace.json   the bench line printed by the traced run

usage: python tools/pmc_summary.py gpurun_out/prof_<tag> <tag>
"""
import csv
import glob
import json
import os
import re
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _find(d, suffix):
    hits = sorted(glob.glob(os.path.join(d, "**", "*" + suffix), recursive=True))
    if not hits:
        raise FileNotFoundError(f"no *{suffix} under {d}")
    return hits[0]


_TOK = [(re.compile(r"DF16b"), "__bf16"), (re.compile(r"Li(-?\d+)E"), None), (re.compile(r"Lb([01])E"), None),
        (re.compile(r"f"), "float"), (re.compile(r"d"), "double"), (re.compile(r"i"), "int"), (re.compile(r"b"), "bool")]


def _demangle_anon(name):
    """c++filt in this image does not know the bf16 mangling (DF16b): decode the template-argument
    lists of our own anonymous-namespace kernels by hand."""
    m = re.match(r"_ZN12_GLOBAL__N_1(\d+)", name)
    if not m:
        return name
    pos = m.end()
    ident = name[pos:pos + int(m.group(1))]
    rest = name[pos + int(m.group(1)):]
    if not rest.startswith("I"):
        return ident
    rest, args = rest[1:], []
    while rest and not rest.startswith("E"):
        for rx, txt in _TOK:
            mm = rx.match(rest)
            if mm:
                args.append(txt if txt else (mm.group(1) if rx.pattern.startswith("Li") else
                                             ("true" if mm.group(1) == "1" else "false")))
                rest = rest[mm.end():]
                break
        else:
            return ident + "<?>"
    return f"{ident}<{', '.join(args)}>"


def short_name(name):
    """'void (anonymous namespace)::gemm_mfma_kernel<__bf16, 0, 0, __bf16>(...)' -> 'gemm_mfma_kernel<__bf16, 0, 0, __bf16>'"""
    if name.startswith("_Z"):
        name = _demangle_anon(name)
    # rocprofv3's own demangler turns the bf16 + bool template pair DF16b Lb1E into
    # "bool _Accum, bool, E" (the false case stays mangled and is decoded above)
    name = name.replace("bool _Accum, bool, E>", "__bf16, true>")
    n = re.sub(r"^void\s+", "", name)
    n = n.replace("(anonymous namespace)::", "")
    depth, out = 0, []
    for ch in n:
        if ch == "(" and depth == 0:
            break
        depth += ch == "<"
        depth -= ch == ">"
        out.append(ch)
    return "".join(out).strip()


def counters(path, counter):
    per = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            if row.get("Counter_Name") != counter:
                continue
            k = short_name(row["Kernel_Name"])
            d = per.setdefault(k, {"dispatches": set(), "sum": 0.0})
            d["dispatches"].add(row["Dispatch_Id"])
            d["sum"] += float(row["Counter_Value"])
    return {k: (len(v["dispatches"]), v["sum"]) for k, v in per.items()}


def main(src, tag):
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    stats = _find(os.path.join(src, "trace"), "kernel_stats.csv")
    shutil.copy(stats, os.path.join(prof, f"{tag}_kernel_stats.csv"))
    bench = os.path.join(src, "bench_trace.json")
    if os.path.exists(bench):
        shutil.copy(bench, os.path.join(prof, f"{tag}_bench_trace.json"))
    fetch = counters(_find(os.path.join(src, "fetch"), "counter_collection.csv"), "FETCH_SIZE")
    write = counters(_find(os.path.join(src, "write"), "counter_collection.csv"), "WRITE_SIZE")
    avg_ns = {}
    with open(stats) as f:
        for row in csv.DictReader(f):
            avg_ns[short_name(row["Name"])] = float(row["AverageNs"])
    out = {}
    for k in sorted(set(fetch) | set(write)):
        nf, sf = fetch.get(k, (0, 0.0))
        nw, sw = write.get(k, (0, 0.0))
        fb = 2.0 * 1024.0 * sf / max(nf, 1)  # FETCH_SIZE is KB; x2 gfx950 correction
        wb = 1024.0 * sw / max(nw, 1)
        out[k] = {"dispatches": max(nf, nw), "fetch_bytes_per_dispatch": fb, "write_bytes_per_dispatch": wb,
                  "traffic_bytes_per_dispatch": fb + wb, "avg_ns_kernel_trace": avg_ns.get(k)}
    meta = {"tag": tag, "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) over "
            "python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline; FETCH_SIZE doubled per the gfx950 "
            "correction", "kernels": out}
    with open(os.path.join(prof, f"{tag}_hbm_traffic.json"), "w") as f:
        json.dump(meta, f, indent=1)
    top = sorted(avg_ns.items(), key=lambda kv: -kv[1])[:5]
    print("wrote profiles/", tag, "top avg kernels:", top)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
