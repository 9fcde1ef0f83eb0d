"""Sum rocprofv3 --pmc counter CSVs (one directory per pass under DIR) per kernel name and print
the per-launch averages for the kernels whose name contains FILTER.
python tools/pmc_kernels.py DIR [FILTER]"""
import collections
import csv
import glob
import os
import sys


def main():
    root = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    launches = collections.defaultdict(set)
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = row["Kernel_Name"]
                if filt not in k:
                    continue
                tot[k][row["Counter_Name"]] += float(row["Counter_Value"])
                launches[(k, row["Counter_Name"])].add(row.get("Dispatch_Id", ""))
    for k, c in sorted(tot.items()):
        print(k[:110])
        for name, v in sorted(c.items()):
            n = max(1, len(launches[(k, name)]))
            print(f"    {name:32s} {v / n:16.4g} per launch ({n} launches)")


if __name__ == "__main__":
    main()
