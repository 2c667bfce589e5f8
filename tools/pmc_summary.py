"""Summarise rocprofv3 outputs of a bench run into profiles/.

  python tools/pmc_summary.py <stats_dir> <fetch_dir> <write_dir> <round> [kernel] [tag]

* <stats_dir>/*_kernel_stats.csv   (rocprofv3 --kernel-trace --stats --output-format csv)
* <fetch_dir>/*_counter_collection.csv (rocprofv3 --pmc FETCH_SIZE, own pass)
* <write_dir>/*_counter_collection.csv (rocprofv3 --pmc WRITE_SIZE, own pass)

FETCH_SIZE / WRITE_SIZE are KiB per dispatch.  gfx950 correction
(MI355X_MICROARCH.md, HBM section): FETCH_SIZE counts half the bytes of a
wide (16 B/lane) coalesced read stream, so it is doubled; WRITE_SIZE is exact
for 16 B/lane stores.  Writes profiles/<round>_pmc_traffic[_<tag>].json and
copies the kernel stats CSV to profiles/<round>_bench_kernel_stats.csv.
"""
import csv
import glob
import json
import os
import shutil
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = "ev_lookup_onehot_kernel"  # bench.py's dominant kernel (argv[5] overrides)
TIMING_LAUNCHES = 20                # bench.py kernel_ms() launches (--kernel-iters default)


def per_dispatch(d, counter):
    f = glob.glob(os.path.join(d, "*_counter_collection.csv"))[0]
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(f))
            if KERNEL in r["Kernel_Name"] and r["Counter_Name"] == counter]
    return vals


def main():
    global KERNEL
    stats_dir, fetch_dir, write_dir, rnd = sys.argv[1:5]
    if len(sys.argv) > 5:
        KERNEL = sys.argv[5]
    tag = ("_" + sys.argv[6]) if len(sys.argv) > 6 else ""
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    st = glob.glob(os.path.join(stats_dir, "*_kernel_stats.csv"))[0]
    shutil.copy(st, os.path.join(prof, "%s_%s_kernel_stats.csv" % (rnd, tag[1:] or "bench")))
    avg_ns = None
    for r in csv.DictReader(open(st)):
        if KERNEL in r["Name"]:
            avg_ns = float(r["AverageNs"])
    # bench.py's HIP-event timing of the dominant kernel is its last
    # TIMING_LAUNCHES dispatches (rotating step batches); the CSV average
    # above also holds the step, check and first-touch launches
    last_ns = None
    tr = glob.glob(os.path.join(stats_dir, "*_kernel_trace.csv"))
    if tr:
        d = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
             for r in csv.DictReader(open(tr[0])) if KERNEL in r["Kernel_Name"]]
        if len(d) >= TIMING_LAUNCHES:
            last_ns = sum(d[-TIMING_LAUNCHES:]) / TIMING_LAUNCHES
    fetch = per_dispatch(fetch_dir, "FETCH_SIZE")
    write = per_dispatch(write_dir, "WRITE_SIZE")
    f_b = statistics.median(fetch) * 1024 * 2   # gfx950: FETCH_SIZE = 1/2 of wide reads
    w_b = statistics.median(write) * 1024
    out = {
        "kernel": KERNEL,
        "source": os.environ.get("PMC_SOURCE") or
                  "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE, separate passes, "
                  "bench.py --no-graph --steps 2 --kernel-iters 3; median over dispatches",
        "fetch_size_kib_raw_median": statistics.median(fetch),
        "write_size_kib_raw_median": statistics.median(write),
        "dispatches": [len(fetch), len(write)],
        "fetch_bytes_corrected": f_b,
        "write_bytes": w_b,
        "bytes_per_launch": f_b + w_b,
        "kernel_avg_ns_rocprof": avg_ns,
        "kernel_avg_ns_rocprof_timing_launches": last_ns,
    }
    json.dump(out, open(os.path.join(prof, "%s_pmc_traffic%s.json" % (rnd, tag)), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
