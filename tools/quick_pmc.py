"""Summary of tools/gpu_quick_pmc.sh passes (the timed render kernel only): kernel time, VALU issue
busy (net of dual issue), VALU instructions, lanes active per VALU instruction, vector-memory and LDS
instructions, TA / TD busy per CU, wave-cycles waiting.
   python tools/quick_pmc.py <dir> [<dir> ...]"""
import csv
import re
import sys
from collections import defaultdict
from pathlib import Path

TIMED = re.compile(r"render_kernel<([^,]+), (true|false), (true|false), false,")
for d in sys.argv[1:]:
    vals, durs = defaultdict(list), []
    for f in Path(d).glob("q*/run_counter_collection.csv"):
        for r in csv.DictReader(f.open()):
            if TIMED.search(r["Kernel_Name"]):
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for f in Path(d).glob("q*/run_kernel_trace.csv"):
        for r in csv.DictReader(f.open()):
            if TIMED.search(r["Kernel_Name"]):
                durs.append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    a = {k: sum(v) / len(v) for k, v in vals.items()}
    cyc = a["GRBM_GUI_ACTIVE"] / 8
    out = {"kernel_ms": sum(durs) / len(durs) / 1e6 if durs else None,
           "valu_busy": 4 * (a["SQ_ACTIVE_INST_VALU"] - a["SQ_ACTIVE_INST_VALU2"]) / (32 * a["SQ_BUSY_CYCLES"]),
           "sq_busy_of_kernel": a["SQ_BUSY_CYCLES"] / 32 / cyc,
           "valu_insts": a["SQ_INSTS_VALU"], "vmem_insts": a["SQ_INSTS_VMEM_RD"], "lds_insts": a["SQ_INSTS_LDS"],
           "salu_insts": a.get("SQ_INSTS_SALU"),
           "lane_util": a["SQ_THREAD_CYCLES_VALU"] / (64 * a["SQ_ACTIVE_INST_VALU"]) if "SQ_THREAD_CYCLES_VALU" in a else None,
           "ta_busy": a["TA_TA_BUSY_sum"] / 256 / cyc if "TA_TA_BUSY_sum" in a else None,
           "td_busy": a["TD_TD_BUSY_sum"] / 256 / cyc if "TD_TD_BUSY_sum" in a else None,
           "wait_inst_any_share": a["SQ_WAIT_INST_ANY"] / a["SQ_WAVE_CYCLES"] if "SQ_WAIT_INST_ANY" in a else None}
    print(d, " ".join(f"{k}={v:.4g}" if isinstance(v, float) else f"{k}={v}" for k, v in out.items()))
