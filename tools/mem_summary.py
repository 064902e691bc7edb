"""Vector-memory pipeline summary of tools/gpu_mem_pmc.sh passes (timed render kernel only):
per-CU TA / TD busy fractions, L1 (TCP) accesses per VMEM instruction and the share that goes to L2.
   python tools/mem_summary.py <dir> [<dir> ...]"""
import csv
import re
import sys
from collections import defaultdict
from pathlib import Path

TIMED = re.compile(r"render_kernel<([^,]+), (true|false), (true|false), false,")
for d in sys.argv[1:]:
    vals = defaultdict(list)
    for f in Path(d).glob("m*/run_counter_collection.csv"):
        for r in csv.DictReader(f.open()):
            if TIMED.search(r["Kernel_Name"]):
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    a = {k: sum(v) / len(v) for k, v in vals.items()}
    cyc = a["GRBM_GUI_ACTIVE"] / 8  # cycles (GRBM_GUI_ACTIVE sums 8 XCDs)
    print(f"{d}: VMEM read instructions {a['SQ_INSTS_VMEM_RD']:.3e}, LDS instructions {a['SQ_INSTS_LDS']:.3e}")
    print(f"  TA busy per CU {a['TA_TA_BUSY_sum'] / 256 / cyc:.3f} (stalled by TC {a['TA_ADDR_STALLED_BY_TC_CYCLES_sum'] / a['TA_TA_BUSY_sum']:.3f} of it)")
    print(f"  TD busy per CU {a['TD_TD_BUSY_sum'] / 256 / cyc:.3f} (stalled by TC {a['TD_TC_STALL_sum'] / a['TD_TD_BUSY_sum']:.3f} of it)")
    print(f"  L1 (TCP) cache accesses per VMEM instruction {a['TCP_TOTAL_CACHE_ACCESSES_sum'] / a['SQ_INSTS_VMEM_RD']:.1f}, "
          f"to L2 per access {a['TCP_TCC_READ_REQ_sum'] / a['TCP_TOTAL_CACHE_ACCESSES_sum']:.4f}")
