"""Per-kernel medians of rocprofv3 --pmc passes (one directory per pass).

  python tools/pmc_counters.py <out.json> <kernel-substring>[|<substring>...] <dir> [<dir> ...]

Reads every <dir>/**/*_counter_collection.csv, keeps the dispatches whose
kernel name contains a substring, and writes, per substring and counter, the
median value per dispatch, the number of dispatches and every dispatch's
value in launch order (a bench run launches a kernel in several roles: the
per-dispatch list tells them apart)."""
import csv
import glob
import json
import os
import statistics
import sys


def main():
    out, subs, dirs = sys.argv[1], sys.argv[2].split("|"), sys.argv[3:]
    res = {}
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*_counter_collection.csv"), recursive=True):
            vals = {}
            for r in csv.DictReader(open(f)):
                for s in subs:
                    if s in r["Kernel_Name"]:
                        key = (s, r["Counter_Name"])
                        vals.setdefault(key, {}).setdefault(r.get("Dispatch_Id", len(vals)), 0.0)
                        vals[key][r.get("Dispatch_Id", len(vals))] += float(r["Counter_Value"])
            for (s, c), per in vals.items():
                v = list(per.values())
                res.setdefault(s, {})[c] = {"median": statistics.median(v), "dispatches": len(v),
                                            "per_dispatch": v,
                                            "pass": os.path.basename(d.rstrip("/"))}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
