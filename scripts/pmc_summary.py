"""Summarise scripts/gpu_pmc.sh counter passes for the conv kernel into JSON.
  python scripts/pmc_summary.py gpurun_out/pmc_<tag> [kernel-substring] [kernel_tag] [kind] > profiles/....json
Per launch (median over the timed launches): duration, effective clock (GRBM_GUI_ACTIVE / 8
XCDs / wall), MFMA-busy fraction, HBM bytes (FETCH_SIZE x2 -- the gfx950 correction of
MI355X_MICROARCH.md -- and WRITE_SIZE, both reported in KiB by rocprofv3), L2 hit rate, LDS
activity and wave-state fractions."""
import csv
import glob
import json
import statistics
import sys

d, key = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "conv_")
vals, durs = {}, []
for f in sorted(glob.glob(f"{d}/p*/pmc_counter_collection.csv")):
    per = {}
    for r in csv.DictReader(open(f)):
        if key not in r["Kernel_Name"]:
            continue
        per.setdefault((r["Counter_Name"], r["Dispatch_Id"]), 0.0)
        per[(r["Counter_Name"], r["Dispatch_Id"])] += float(r["Counter_Value"])
    for (c, _), v in per.items():
        vals.setdefault(c, []).append(v)
for f in sorted(glob.glob(f"{d}/p*/pmc_kernel_trace.csv")):
    for r in csv.DictReader(open(f)):
        if key in r["Kernel_Name"]:
            durs.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
med = {c: statistics.median(v[2:] if len(v) > 4 else v) for c, v in vals.items()}
dur = statistics.median(durs[2:] if len(durs) > 4 else durs)
out = {"source": d, "kernel_match": key, "launch_s": dur}
if len(sys.argv) > 3:                      # the kernel the bench's roofline names (bench.pmc_traffic checks it)
    out["kernel_tag"] = sys.argv[3]
if len(sys.argv) > 4:                      # which of its launch kinds (scripts/conv_one.py KIND)
    out["kind"] = sys.argv[4]
if "GRBM_GUI_ACTIVE" in med:
    clk = med["GRBM_GUI_ACTIVE"] / 8 / dur
    out["clock_ghz"] = round(clk / 1e9, 3)
    if "SQ_VALU_MFMA_BUSY_CYCLES" in med:
        out["mfma_busy"] = round(med["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024 / (dur * clk), 3)
    if "SQ_LDS_IDX_ACTIVE" in med:
        out["lds_active_per_cu_cycle"] = round(med["SQ_LDS_IDX_ACTIVE"] / 256 / (dur * clk), 3)
if "FETCH_SIZE" in med:
    out["hbm_read_bytes"] = med["FETCH_SIZE"] * 1024 * 2
if "WRITE_SIZE" in med:
    out["hbm_write_bytes"] = med["WRITE_SIZE"] * 1024
if "FETCH_SIZE" in med and "WRITE_SIZE" in med:
    out["hbm_bytes"] = out["hbm_read_bytes"] + out["hbm_write_bytes"]
if "TCC_HIT_sum" in med:
    out["l2_hit"] = round(med["TCC_HIT_sum"] / (med["TCC_HIT_sum"] + med["TCC_MISS_sum"]), 3)
wc = med.get("SQ_WAVE_CYCLES")
if wc:
    for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
        if c in med:
            out[c.lower() + "_frac"] = round(med[c] / wc, 3)
out["counters"] = med
print(json.dumps(out, indent=1))
