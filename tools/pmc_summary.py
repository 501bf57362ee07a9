"""Summarise a tools/profile.sh run into profiles/<tag>/.

Copies the kernel-trace stats CSV and derives, for the engine kernel, the
average dispatch duration and HBM traffic per launch from the PMC passes:
  FETCH_SIZE, WRITE_SIZE are in KiB per dispatch (rocprofv3, gfx950).
  MI355X_MICROARCH.md §HBM: FETCH_SIZE reads exactly 1/2 of the bytes of a wide
  (16 B/lane) coalesced stream; other widths are uncalibrated.  The QP kernels
  stage their inputs with 16-B loads (mpcqp_form.h::form_stage), so the x2
  correction applies to them; the raw figure is reported as well.
"""
import csv
import glob
import json
import os
import shutil
import sys

KERNEL = "mpcqp"


def rows(pattern):
    out = []
    for f in glob.glob(pattern, recursive=True):
        with open(f) as fh:
            out.extend(csv.DictReader(fh))
    return out


def kname(name):
    for k in ("mpcqp_kernel_128", "mpcqp_kernel_96", "mpcqp_kernel_64", "mpcqp_kernel_ipm", "mpcqp_order_kernel",
              "mpcqp_plan_kernel", "mpcqp_stance_torque_kernel"):
        if k in name:
            return k
    return name


def counter(run_dir, name, kernel):
    """Per-dispatch values of one counter for one engine kernel."""
    vals = []
    for r in rows(os.path.join(run_dir, "**", "*counter_collection.csv")):
        if kname(r.get("Kernel_Name", "")) == kernel and r.get("Counter_Name") == name:
            vals.append(float(r["Counter_Value"]))
    return vals


def main():
    src, dst = sys.argv[1], sys.argv[2]
    args = sys.argv[3:]
    os.makedirs(dst, exist_ok=True)
    for f in glob.glob(os.path.join(src, "kt", "**", "*stats.csv"), recursive=True):
        shutil.copy(f, os.path.join(dst, os.path.basename(f)))
    stats = rows(os.path.join(src, "kt", "**", "*kernel_stats.csv"))
    kernels = {}
    for r in stats:
        if KERNEL in r["Name"]:
            kernels[kname(r["Name"])] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                                         "total_ns": float(r["TotalDurationNs"])}
    dominant = max(kernels, key=lambda k: kernels[k]["total_ns"]) if kernels else None
    bench = {}
    try:
        with open(os.path.join(src, "bench_kt.json")) as fh:
            bench = json.loads(fh.read().strip().splitlines()[-1])
    except Exception:
        pass
    cfg = "config2"
    for i, a in enumerate(args):
        if a == "--config" and i + 1 < len(args):
            cfg = args[i + 1]
    batch = bench.get("config", {}).get("batch_per_gpu")
    per_kernel = {}
    for k, st in kernels.items():
        fetch = counter(os.path.join(src, "fetch"), "FETCH_SIZE", k)
        write = counter(os.path.join(src, "write"), "WRITE_SIZE", k)
        fk = sum(fetch) / len(fetch) if fetch else None
        wk = sum(write) / len(write) if write else None
        per_kernel[k] = dict(st, fetch_kib_per_launch_raw=fk, write_kib_per_launch=wk,
                             hbm_bytes_per_launch=(2 * fk * 1024 + wk * 1024) if fk is not None and wk is not None
                             else None)
    dom = per_kernel.get(dominant, {})
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "pympc-quadruped_amd"))
    from mpcqp import _lib
    entry = {
        "batch": batch,
        "lib_sha256": _lib.lib_sha256(),   # the build these counters belong to (bench.py checks it)
        "profile_dir": dst,
        "dominant_kernel": dominant,
        "kernel_avg_ns_rocprof": dom.get("avg_ns"),
        "kernel_ms_avg_bench_events": bench.get("kernel_ms_avg"),
        "hbm_bytes_per_launch": dom.get("hbm_bytes_per_launch"),
        "kernels": per_kernel,
        "note": "FETCH_SIZE x2 per MI355X_MICROARCH.md (16-B/lane stream calibration; the QP kernels stage inputs with 16-B loads)",
    }
    path = os.path.join(dst, "pmc_traffic.json")
    data = {}
    if os.path.exists(path):
        with open(path) as fh:
            data = json.load(fh)
    data[cfg] = entry
    with open(path, "w") as fh:
        json.dump(data, fh, indent=2)
    print(json.dumps({cfg: entry}))


if __name__ == "__main__":
    main()
