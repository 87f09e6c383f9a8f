"""Medians per kernel of the PMC passes of tools/pmc_kernel.sh, with derived
figures: VALU instructions per wave, the fraction of wave cycles waiting,
fp64 share of the VALU instructions, LDS bank conflicts per LDS instruction,
and TA busy per XCD (TA_BUSY_avr / (GRBM_GUI_ACTIVE / 8 XCDs)).
usage: python tools/sq_json.py gpurun_out/<tag>   (reads <tag>_{A,B,C,D}/)"""
import collections
import csv
import json
import statistics
import sys
from pathlib import Path

base = Path(sys.argv[1])
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for p in "ABCD":
    f = Path(f"{base}_{p}") / "run_counter_collection.csv"
    if not f.exists():
        continue
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].split("(")[0]
        agg[name][(p, r["Counter_Name"])].append(float(r["Counter_Value"]))
out = {}
for k, cs in agg.items():
    m = {}
    for (p, c), v in cs.items():
        key = c if c != "GRBM_GUI_ACTIVE" else f"GRBM_GUI_ACTIVE_{p}"
        m[key] = statistics.median(v)
    w = m.get("SQ_WAVES")
    if w:
        m["valu_per_wave"] = m.get("SQ_INSTS_VALU", 0.0) / w
    if m.get("SQ_WAVE_CYCLES"):
        m["wait_any_frac"] = m.get("SQ_WAIT_ANY", 0.0) / m["SQ_WAVE_CYCLES"]
    f64 = sum(m.get(c, 0.0) for c in ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64",
                                      "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_TRANS_F64"))
    if m.get("SQ_INSTS_VALU"):
        m["fp64_share_of_valu"] = f64 / m["SQ_INSTS_VALU"]
    if m.get("SQ_INSTS_LDS"):
        m["lds_bank_conflict_per_lds_inst"] = m.get("SQ_LDS_BANK_CONFLICT", 0.0) / m["SQ_INSTS_LDS"]
    if m.get("GRBM_GUI_ACTIVE_D") and "TA_BUSY_avr" in m:
        m["ta_busy_frac_per_xcd"] = m["TA_BUSY_avr"] / (m["GRBM_GUI_ACTIVE_D"] / 8.0)
    out[k] = m
out["note"] = ("medians over the dispatches of the run; rocprofv3 --pmc passes A-D "
               "(tools/pmc_kernel.sh), kernel-include regex, no trace domains; "
               "TA fraction = TA_BUSY_avr / (GRBM_GUI_ACTIVE / 8 XCDs)")
print(json.dumps(out, indent=1))
