#!/usr/bin/env python3
"""Per-kernel summary of rocprofv3 counter databases (rocpd sqlite, ROCm 7.x) or counter CSVs.

    python tools/pmc_summary.py gpurun_out/pmc_a/run_results.db [more.db ...] [--match gemm_h3p] [--top 20]

Counters of several single-pass runs of the same program are joined by kernel name (each pass is
its own run: rocprofv3 does not split counters over passes).  Per kernel: dispatches, mean
duration, the mean of every counter per dispatch, and derived columns when their inputs exist:
bf16 / fp16 MFMA TF/s (512 FLOP per MOPS unit), MFMA busy % of the dispatch's SQ busy cycles, LDS
bank-conflict % of LDS-active cycles, L2 hit %, wait % of wave cycles.
"""
import argparse
import collections
import re
import sqlite3


def short(name, n=70):
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"\(.*", "", name)
    return name if len(name) <= n else name[:n - 3] + "..."


def load(db):
    if db.endswith(".csv"):  # rocprofv3 --output-format csv: run_counter_collection.csv
        import csv

        per = collections.defaultdict(lambda: collections.defaultdict(list))
        durs = collections.defaultdict(dict)
        for r in csv.DictReader(open(db)):
            name, disp = r["Kernel_Name"], int(r["Dispatch_Id"])
            per[name][r["Counter_Name"]].append((disp, float(r["Counter_Value"])))
            durs[name][disp] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        return per, durs
    c = sqlite3.connect(db)
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    durs = collections.defaultdict(dict)
    for name, disp, counter, value, dur in c.execute(
            "select kernel_name, dispatch_id, counter_name, value, duration from counters_collection"):
        per[name][counter].append((disp, value))
        durs[name][disp] = dur
    return per, durs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dbs", nargs="+")
    ap.add_argument("--match", default=None)
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--raw", action="store_true", help="also print every counter's mean per dispatch")
    a = ap.parse_args()
    counters = collections.defaultdict(dict)  # kernel -> counter -> mean per dispatch
    ndisp, dur = {}, {}
    for db in a.dbs:
        per, durs = load(db)
        for k, cs in per.items():
            if a.match and not re.search(a.match, k):
                continue
            for cn, vals in cs.items():
                bydisp = collections.defaultdict(float)
                for d, v in vals:
                    bydisp[d] += v
                counters[k][cn] = sum(bydisp.values()) / len(bydisp)
            ndisp[k] = max(ndisp.get(k, 0), len(durs[k]))
            dur.setdefault(k, []).extend(durs[k].values())
    rows = []
    for k, cs in counters.items():
        d = sum(dur[k]) / len(dur[k])  # ns
        row = {"kernel": short(k), "n": ndisp[k], "us": d / 1000.0}
        if "SQ_INSTS_VALU_MFMA_MOPS_BF16" in cs:
            row["bf16 TF/s"] = cs["SQ_INSTS_VALU_MFMA_MOPS_BF16"] * 512 / d / 1000.0
        if "SQ_INSTS_VALU_MFMA_MOPS_F16" in cs:
            row["f16 TF/s"] = cs["SQ_INSTS_VALU_MFMA_MOPS_F16"] * 512 / d / 1000.0
        if "SQ_VALU_MFMA_BUSY_CYCLES" in cs and "SQ_BUSY_CYCLES" in cs and cs["SQ_BUSY_CYCLES"]:
            row["mfma busy/SQ busy %"] = 100.0 * cs["SQ_VALU_MFMA_BUSY_CYCLES"] / (cs["SQ_BUSY_CYCLES"] * 4 * 4)
        if "SQ_INSTS_LDS" in cs and "GRBM_GUI_ACTIVE" in cs and cs["GRBM_GUI_ACTIVE"]:
            # LDS instructions per CU per cycle (256 CUs; GRBM_GUI_ACTIVE sums the 8 XCDs' cycles)
            row["lds inst/CU/kclk"] = 1000.0 * cs["SQ_INSTS_LDS"] / 256 / (cs["GRBM_GUI_ACTIVE"] / 8)
        if "SQ_LDS_IDX_ACTIVE" in cs and cs.get("SQ_BUSY_CYCLES"):
            row["lds active/SQ busy %"] = 100.0 * cs["SQ_LDS_IDX_ACTIVE"] / cs["SQ_BUSY_CYCLES"]
        if "SQ_LDS_BANK_CONFLICT" in cs and cs.get("SQ_LDS_IDX_ACTIVE"):
            row["lds conflict %"] = 100.0 * cs["SQ_LDS_BANK_CONFLICT"] / cs["SQ_LDS_IDX_ACTIVE"]
        if "TCC_HIT_sum" in cs and (cs["TCC_HIT_sum"] + cs.get("TCC_MISS_sum", 0)):
            row["L2 hit %"] = 100.0 * cs["TCC_HIT_sum"] / (cs["TCC_HIT_sum"] + cs.get("TCC_MISS_sum", 0))
        if "SQ_WAVE_CYCLES" in cs and cs["SQ_WAVE_CYCLES"]:
            for w in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
                if w in cs:
                    row[w.replace("SQ_", "").lower() + " %"] = 100.0 * cs[w] / cs["SQ_WAVE_CYCLES"]
        if "GRBM_GUI_ACTIVE" in cs:
            row["clock GHz"] = cs["GRBM_GUI_ACTIVE"] / 8 / d
        if a.raw:
            row.update({c: float(v) for c, v in cs.items()})
        rows.append(row)
    rows.sort(key=lambda r: -r["us"] * r["n"])
    cols = ["kernel", "n", "us"] + sorted({c for r in rows for c in r} - {"kernel", "n", "us"})
    print("| " + " | ".join(cols) + " |")
    print("|" + "---|" * len(cols))
    for r in rows[:a.top]:
        print("| " + " | ".join(("%.1f" % r[c]) if isinstance(r.get(c), float) else str(r.get(c, "")) for c in cols)
              + " |")


if __name__ == "__main__":
    main()
