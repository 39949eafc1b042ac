#!/usr/bin/env python3
"""Summarise a tools/gpu_session.sh prof+pmc run into profiles/ (committed evidence).

  python tools/summarize_prof.py r01          (config 2: dirs prof, pmc1..pmc4)
  python tools/summarize_prof.py r01c3 _c3    (config 3: dirs prof_c3, pmc1_c3..pmc4_c3)
writes
  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (copied)
  profiles/<tag>_pmc_summary.json   per-kernel counters per launch (VALU, HBM bytes)
  profiles/pmc_traffic.json         HBM bytes/launch per kernel (config 2 run only)
bench.py reads <tag>_pmc_summary.json of the config it runs (PMC_SUMMARY there).
FETCH_SIZE is doubled: on gfx950 it reports half the bytes of a wide coalesced read
(/opt/skills/guides/MI355X_MICROARCH.md, HBM section); both are in KB.
"""
import collections
import csv
import json
import os
import re
import shutil
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")


def short(name: str) -> str:
    m = re.search(r"(k_scan<[^>]*>|k_reduce|__amd_rocclr_\w+)", name)
    return m.group(1) if m else name[:60]


def load_pmc(d):
    """{kernel: {counter: {dispatch: value}}} of one --pmc pass."""
    path = os.path.join(OUT, d, "pmc_counter_collection.csv")
    if not os.path.exists(path):
        return {}
    vals = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(float)))
    for r in csv.DictReader(open(path)):
        vals[short(r["Kernel_Name"])][r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    return vals


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
    sfx = sys.argv[2] if len(sys.argv) > 2 else ""
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    stats = os.path.join(OUT, "prof" + sfx, "bench_kernel_stats.csv")
    if os.path.exists(stats):
        shutil.copy(stats, os.path.join(prof, f"{tag}_kernel_stats.csv"))
    # build id of the library the box ran (tools/gpu_session.sh writes it at session
    # start); bench.py uses these counters only while the library has the same id
    bid_path = os.path.join(OUT, "build_id.txt")
    build_id = open(bid_path).read().strip() if os.path.exists(bid_path) else None
    summary = {"tag": tag, "build_id": build_id, "kernels": {}}
    traffic = {"source": f"profiles/{tag}_pmc_summary.json", "kernels": {}}
    # per launch = the MEDIAN over the profiled dispatches of a kernel (round 3; rounds 1-2
    # took the mean): one of three config-2 launches once read 79 MB of FETCH_SIZE against
    # 2.3 MB for the other two (profiles/r03_pmc_summary.json keeps the max beside it)
    merged = collections.defaultdict(dict)
    maxes = collections.defaultdict(dict)
    launches = {}
    for d in ("pmc1", "pmc2", "pmc3", "pmc4"):
        for k, cs in load_pmc(d + sfx).items():
            for c, per in cs.items():
                xs = sorted(per.values())
                merged[k][c] = statistics.median(xs)
                maxes[k][c] = xs[-1]
                launches[k] = len(xs)
    for k, cs in merged.items():
        e = {"launches_profiled": launches.get(k), "per_launch": cs, "per_launch_max": maxes[k]}
        if "FETCH_SIZE" in cs or "WRITE_SIZE" in cs:
            hbm = (2.0 * cs.get("FETCH_SIZE", 0.0) + cs.get("WRITE_SIZE", 0.0)) * 1024.0
            e["hbm_bytes_per_launch"] = hbm
            traffic["kernels"][k.lower()] = {"hbm_bytes_per_launch": hbm}
        if "GRBM_GUI_ACTIVE" in cs and "SQ_INSTS_VALU" in cs:
            cycles = cs["GRBM_GUI_ACTIVE"] / 8.0  # summed over the 8 XCDs
            e["gpu_cycles_per_launch"] = cycles
            # lane-instructions per CU per clock (256 CUs, 64 lanes): 64 = VOP3 issue peak
            e["valu_lane_ops_per_cu_per_clk"] = cs["SQ_INSTS_VALU"] * 64.0 / 256.0 / cycles
            if "SQ_INSTS_VALU_INT32" in cs:
                e["int32_valu_fraction"] = cs["SQ_INSTS_VALU_INT32"] / cs["SQ_INSTS_VALU"]
        summary["kernels"][k] = e
    json.dump(summary, open(os.path.join(prof, f"{tag}_pmc_summary.json"), "w"), indent=1)
    if not sfx:
        json.dump(traffic, open(os.path.join(prof, "pmc_traffic.json"), "w"), indent=1)
    print(json.dumps(summary, indent=1)[:3000])


if __name__ == "__main__":
    main()
