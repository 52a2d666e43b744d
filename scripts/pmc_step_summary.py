"""Summarise scripts/gpu_pmc_step.sh counter passes per kernel (all kernels of the profiled step).
  python scripts/pmc_step_summary.py gpurun_out/pmcstep_<tag> [top] > profiles/...json
Per kernel (grouped by the full kernel name; medians over its dispatches in the LAST half of each pass,
i.e. the timed step rather than the warm-up): dispatches per pass, duration, effective clock
(GRBM_GUI_ACTIVE / 8 XCDs / wall), MFMA-busy fraction (SQ_VALU_MFMA_BUSY_CYCLES / 1024 SIMDs), HBM bytes
(FETCH_SIZE x 2 -- the gfx950 correction of MI355X_MICROARCH.md -- plus WRITE_SIZE, rocprofv3 reports both
in KiB), achieved HBM bandwidth, L2 hit rate, wave-state fractions, VALU / LDS instructions per wave."""
import csv
import glob
import json
import statistics
import sys


def short(name):
    return name.replace("(anonymous namespace)::", "").replace("void ", "")[:160]


def main():
    d = sys.argv[1]
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    vals, durs, ndisp = {}, {}, {}
    for f in sorted(glob.glob(f"{d}/p*/pmc_counter_collection.csv")):
        per = {}
        order = []
        for r in csv.DictReader(open(f)):
            key = (r["Kernel_Name"], r["Dispatch_Id"])
            if key not in per:
                order.append(key)
            per.setdefault(key, {}).setdefault(r["Counter_Name"], 0.0)
            per[key][r["Counter_Name"]] += float(r["Counter_Value"])
        half = order[len(order) // 2:]          # the timed step (the first half is the warm-up step)
        for key in half:
            for c, v in per[key].items():
                vals.setdefault(key[0], {}).setdefault(c, []).append(v)
    for f in sorted(glob.glob(f"{d}/p*/pmc_kernel_trace.csv")):
        rows = list(csv.DictReader(open(f)))
        rows = rows[len(rows) // 2:]
        cnt = {}
        for r in rows:
            durs.setdefault(r["Kernel_Name"], []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
            cnt[r["Kernel_Name"]] = cnt.get(r["Kernel_Name"], 0) + 1
        for k, v in cnt.items():
            ndisp[k] = max(ndisp.get(k, 0), v)
    out = []
    for k, ds in durs.items():
        dur = statistics.median(ds)
        med = {c: statistics.median(v) for c, v in vals.get(k, {}).items()}
        e = {"kernel": short(k), "dispatches_per_step": ndisp.get(k), "launch_us": round(dur * 1e6, 2),
             "total_us_per_step": round(dur * 1e6 * ndisp.get(k, 0), 1)}
        clk = None
        if "GRBM_GUI_ACTIVE" in med and dur > 0:
            clk = med["GRBM_GUI_ACTIVE"] / 8 / dur
            e["clock_ghz"] = round(clk / 1e9, 3)
            if "SQ_VALU_MFMA_BUSY_CYCLES" in med:
                e["mfma_busy"] = round(med["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024 / (dur * clk), 3)
            if "SQ_LDS_IDX_ACTIVE" in med:
                e["lds_active_per_cu_cycle"] = round(med["SQ_LDS_IDX_ACTIVE"] / 256 / (dur * clk), 3)
        if "FETCH_SIZE" in med:
            e["hbm_read_bytes"] = med["FETCH_SIZE"] * 1024 * 2
        if "WRITE_SIZE" in med:
            e["hbm_write_bytes"] = med["WRITE_SIZE"] * 1024
        if "FETCH_SIZE" in med and "WRITE_SIZE" in med:
            e["hbm_bytes"] = e["hbm_read_bytes"] + e["hbm_write_bytes"]
            e["hbm_tb_s"] = round(e["hbm_bytes"] / dur / 1e12, 3)
        if "TCC_HIT_sum" in med and med["TCC_HIT_sum"] + med.get("TCC_MISS_sum", 0) > 0:
            e["l2_hit"] = round(med["TCC_HIT_sum"] / (med["TCC_HIT_sum"] + med["TCC_MISS_sum"]), 3)
        wc = med.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
                if c in med:
                    e[c.lower() + "_frac"] = round(med[c] / wc, 3)
        waves = med.get("SQ_WAVES")
        if waves:
            for c in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR"):
                if c in med:
                    e[c.lower() + "_per_wave"] = round(med[c] / waves, 1)
            if "SQ_LDS_BANK_CONFLICT" in med and med.get("SQ_LDS_IDX_ACTIVE"):
                e["lds_bank_conflict_frac"] = round(med["SQ_LDS_BANK_CONFLICT"] / med["SQ_LDS_IDX_ACTIVE"], 3)
        e["counters"] = {c: round(v, 1) for c, v in med.items()}
        out.append(e)
    out.sort(key=lambda e: -e["total_us_per_step"])
    print(json.dumps({"source": d, "kernels": out[:top]}, indent=1))


if __name__ == "__main__":
    main()
