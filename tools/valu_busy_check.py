"""Checks the counter-based VALU busy fraction (tools/pmc_summary.py: 4 x (SQ_ACTIVE_INST_VALU -
SQ_ACTIVE_INST_VALU2) / (32 x SQ_BUSY_CYCLES)) on tools/valu_rate.hip, whose kernels issue one
instruction kind back to back: at 8 waves per SIMD every kind should read close to 1, and only the
kinds that dual-issue show SQ_ACTIVE_INST_VALU2.
  rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_BUSY_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE \
      --kernel-trace --output-format csv -d <dir> -o run -- tools/build/valu_rate
  python tools/valu_busy_check.py <dir>/run_counter_collection.csv
"""
import csv
import re
import sys
from collections import defaultdict

NAMES = ["v_fma_f32", "v_add_f64", "v_mul_f64", "v_fma_f64", "v_rcp_f64", "v_add_f32", "v_mul_f32", "v_xor_b32",
         "v_rcp_f32", "v_pk_fma_f32", "v_pk_add_f32", "v_min_f32", "v_max3_f32", "v_cndmask_b32", "v_min_i32",
         "v_max_u32", "v_med3_f32", "v_min3_i32", "v_min_f64", "v_cmp_lt_f32", "v_bfe_u32", "v_lshl_or_b32",
         "v_mul_lo_u32", "v_mul_hi_u32", "v_mad_u32_u24", "v_cvt_f32_u32", "v_cvt_f64_u32", "v_rsq_f64",
         "v_sqrt_f64", "v_cmp_lt_f64", "v_mov_b32", "v_add_u32"]


def main():
    rows = defaultdict(dict)
    for r in csv.DictReader(open(sys.argv[1])):
        k = (int(r["Dispatch_Id"]), r["Kernel_Name"])
        rows[k][r["Counter_Name"]] = rows[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    by_kind = defaultdict(list)
    for (_, name), c in sorted(rows.items()):
        m = re.search(r"rate_kernel<(\d+)", name)
        if m:
            by_kind[int(m.group(1))].append(c)
    print(f"{'instruction':15s} {'waves/SIMD':>10s} {'quads/inst':>10s} {'dual/inst':>9s} {'VALU busy':>9s}")
    for kind, launches in sorted(by_kind.items()):
        # per kind: (warm-up, timed) at 1, 2, 4 and 8 waves per SIMD; the timed ones at 1 and 8
        for waves, c in ((1, launches[1]), (8, launches[-1])):
            simd = 32 * c["SQ_BUSY_CYCLES"]
            busy = 4 * (c["SQ_ACTIVE_INST_VALU"] - c["SQ_ACTIVE_INST_VALU2"]) / simd
            print(f"{NAMES[kind]:15s} {waves:10d} {c['SQ_ACTIVE_INST_VALU'] / c['SQ_INSTS_VALU']:10.2f} "
                  f"{c['SQ_ACTIVE_INST_VALU2'] / c['SQ_INSTS_VALU']:9.2f} {busy:9.3f}")


if __name__ == "__main__":
    main()
