"""Per-kernel summary of rocprofv3 --pmc passes (run_counter_collection.csv files): the
counters averaged over a kernel's dispatches, with the derived figures used in DESIGN:
MFMA busy fraction (SQ_VALU_MFMA_BUSY_CYCLES over the launch's SIMD-cycles at 2.4 GHz x
1024 SIMDs, the launch time from a kernel_stats.csv of the same command), wait shares of
SQ_WAVE_CYCLES, LDS bank-conflict share, and L2-miss bytes per launch (gfx950:
2 FETCH_SIZE KB + WRITE_SIZE KB, MI355X_MICROARCH.md's HBM/rocprofv3 correction).
Usage: python tools/pmc_summary.py KERNEL_STATS.csv PASS.csv [PASS.csv ...] > summary.json"""
import collections
import csv
import json
import re
import sys


def short(name):
    m = re.search(r"rsx::(?:sf::)?(\w+)(<[^>]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:60]


def main():
    stats = {short(r["Name"]): float(r["AverageNs"]) for r in csv.DictReader(open(sys.argv[1]))}
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    meta = {}
    for f in sys.argv[2:]:
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            meta[k] = {"grid": int(float(r["Grid_Size"])), "workgroup": int(float(r["Workgroup_Size"])),
                       "lds_bytes": int(float(r["LDS_Block_Size"])), "vgpr": int(float(r["VGPR_Count"])),
                       "agpr": int(float(r["Accum_VGPR_Count"]))}
    out = {}
    for k, d in sorted(acc.items()):
        c = {n: sum(v) / len(v) for n, v in d.items()}
        e = dict(meta[k], counters=c)
        ns = stats.get(k)
        if ns:
            e["avg_launch_us"] = ns / 1e3
            simd_cycles = ns * 1e-9 * 2.4e9 * 1024
            if "SQ_VALU_MFMA_BUSY_CYCLES" in c:
                e["mfma_busy_frac"] = c["SQ_VALU_MFMA_BUSY_CYCLES"] / simd_cycles
        wc = c.get("SQ_WAVE_CYCLES")
        if wc:
            for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if n in c:
                    e[n.lower() + "_share"] = c[n] / wc
        if c.get("SQ_LDS_IDX_ACTIVE"):
            e["lds_conflict_share"] = c.get("SQ_LDS_BANK_CONFLICT", 0.0) / c["SQ_LDS_IDX_ACTIVE"]
        if "FETCH_SIZE" in c or "WRITE_SIZE" in c:
            e["l2_miss_bytes_per_launch"] = (2 * c.get("FETCH_SIZE", 0.0) + c.get("WRITE_SIZE", 0.0)) * 1024
        if "SQ_WAVES" in c:
            e["waves_per_simd"] = c["SQ_WAVES"] / 1024
        out[k] = e
    json.dump(out, sys.stdout, indent=1)


if __name__ == "__main__":
    main()
