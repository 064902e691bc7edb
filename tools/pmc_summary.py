"""Summarise the rocprofv3 PMC passes of tools/gpu_pmc.sh (<dir>/p*/run_counter_collection.csv)
into the per-launch counter JSON bench.py reads (profiles/pmc_latest.json for config 2).

Per the MI355X_MICROARCH guide's HBM section: FETCH_SIZE (KB) under-reads wide coalesced reads on
gfx950 by 2x, so HBM read bytes = 2 * FETCH_SIZE * 1024; WRITE_SIZE (KB) is taken as is. Each
counter group ran in its own rocprofv3 --pmc pass. Values are averaged over the launches of the
timed render kernel (template COUNT = false; the instrumented pass is excluded).

VALU issue. SQ_BUSY_CYCLES sums busy cycles over the 32 SQs (8 XCDs x 4 shader engines), so the
chip's SIMD-cycles are 32 x SQ_BUSY_CYCLES (1024 SIMDs); the model-free cross-check is the
SIMD-cycles from GRBM_GUI_ACTIVE (summed over 8 XCDs: 1024 x GRBM_GUI_ACTIVE / 8), which also gives
the effective clock GRBM_GUI_ACTIVE / 8 / kernel time. Issue cycles two ways:
  valu_issue_frac_model     2 cycles per wave64 VALU instruction, 4 per f64 one (the textbook
                            SIMD-32 model; the round-2 figure)
  valu_issue_frac_measured  each instruction class (SQ_INSTS_VALU_* counters, pass 5) at the
                            SIMD cycles per wave64 instruction tools/valu_rate.hip measured on the
                            MI355X (profiles/r03_v3/valu_rate.json: wall time x shader clock over
                            each SIMD's instructions, 8 waves per SIMD, loop overhead included):
                            f32 add / mul / fma and int32 2.30-2.41 (nominal 2), f64 add / mul /
                            fma 4.15-4.18 (nominal 4), f32 transcendental 8.16 (8), f64
                            transcendental 16.16 (16). The summary uses the nominal values the
                            measurement confirms; CVT and int64 count as f64-class (4), every
                            other VALU instruction (moves, selects, compares, packed f32) as 2.
  valu_busy_frac            (when pass 6 ran; then also valu_issue_frac) model-free: the quad-cycles
                            the waves issue VALU work (SQ_ACTIVE_INST_VALU, summed over waves)
                            less the quad-cycles two waves issued together (SQ_ACTIVE_INST_VALU2,
                            gfx950 dual issue), x 4, over the SIMD cycles. The class model above
                            undercounts: most "other" instructions (v_cndmask, v_cmp, v_min / max,
                            v_bfe, packed f32, conversions) take a full quad-cycle (4.1-4.3 cycles,
                            profiles/r03_v3/valu_rate_ext.json); only f32 add / mul / fma, v_mov,
                            v_add_u32, v_xor pair up (2.3).

usage: python tools/pmc_summary.py <pmc dir> <out.json> [workload]
The workload key defaults to config.workload of <dir>/bench_p1.json (the bench line of pass 1);
the summary records bench.kernel_source_sha() (the loaded library's build info: its switches and
the sha of the sources it was compiled from) and the git commit of that build, so bench.py only
uses counters collected on the build it is timing; a library built from uncommitted sources is
refused (tools/gpu_pmc.sh checks before collecting, this script again).
"""
import csv
import json
import re
import sys
from collections import defaultdict
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from bench import build_stamp, kernel_source_sha  # noqa: E402

TIMED = re.compile(r"render_kernel<([^,]+), (true|false), (true|false), false,")


def main():
    src, out = Path(sys.argv[1]), Path(sys.argv[2])
    if len(sys.argv) > 3:
        workload = sys.argv[3]
    else:
        workload = json.loads((src / "bench_p1.json").read_text().strip().splitlines()[-1])["config"]["workload"]
    vals = defaultdict(list)
    durs = []
    names = set()
    for f in sorted(src.glob("p*/run_counter_collection.csv")):
        for r in csv.DictReader(f.open()):
            name = r["Kernel_Name"].removeprefix("void ")
            if TIMED.search(name):
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
                names.add(name.split("(")[0])
    for f in sorted(src.glob("p*/run_kernel_trace.csv")):
        for r in csv.DictReader(f.open()):
            if TIMED.search(r["Kernel_Name"]):
                durs.append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    if len(names) > 1:
        raise SystemExit(f"several timed kernel instances under {src}: {sorted(names)}")
    if not vals:
        raise SystemExit(f"no timed render_kernel rows under {src}")
    avg = {k: sum(v) / len(v) for k, v in vals.items()}
    stamp = build_stamp()
    if stamp["git_dirty"]:
        raise SystemExit(f"library built from uncommitted sources ({stamp['build_info']}): not summarised")
    res = {"workload": workload, "kernel": names.pop(), "kernel_source_sha": kernel_source_sha(),
           "git_commit": stamp["git_commit"], "git_dirty": False, "source_sha": stamp["source_sha"],
           "build_info": stamp["build_info"], "launches": {k: len(v) for k, v in vals.items()}}
    if durs:
        res["kernel_ns_under_pmc"] = sum(durs) / len(durs)
    res.update({k: avg[k] for k in sorted(avg)})
    if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
        res["FETCH_SIZE_KB"] = avg["FETCH_SIZE"]
        res["WRITE_SIZE_KB"] = avg["WRITE_SIZE"]
        res["hbm_bytes_per_launch"] = int(round(2 * avg["FETCH_SIZE"] * 1024 + avg["WRITE_SIZE"] * 1024))
        res["correction"] = ("MI355X_MICROARCH.md HBM: FETCH_SIZE reads 1/2 of wide coalesced reads on "
                             "gfx950 -> x2; WRITE_SIZE taken as is; separate --pmc passes (tools/gpu_pmc.sh)")
    if "TCC_HIT_sum" in avg and "TCC_MISS_sum" in avg:
        res["l2_hit_rate"] = avg["TCC_HIT_sum"] / max(1.0, avg["TCC_HIT_sum"] + avg["TCC_MISS_sum"])
    f64 = ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_TRANS_F64")
    if "SQ_INSTS_VALU" in avg and "SQ_BUSY_CYCLES" in avg and all(k in avg for k in f64):
        n64 = sum(avg[k] for k in f64)
        res["valu_issue_cycles_model"] = 2 * avg["SQ_INSTS_VALU"] + 2 * n64
        res["simd_cycles"] = 32 * avg["SQ_BUSY_CYCLES"]
        res["valu_issue_frac_model"] = res["valu_issue_cycles_model"] / res["simd_cycles"]
        res["valu_insts_per_simd_cycle"] = avg["SQ_INSTS_VALU"] / res["simd_cycles"]
        cls = {"SQ_INSTS_VALU_ADD_F32": 2, "SQ_INSTS_VALU_MUL_F32": 2, "SQ_INSTS_VALU_INT32": 2,
               "SQ_INSTS_VALU_FMA_F32": 2, "SQ_INSTS_VALU_CVT": 4, "SQ_INSTS_VALU_TRANS_F32": 8,
               "SQ_INSTS_VALU_ADD_F64": 4, "SQ_INSTS_VALU_MUL_F64": 4, "SQ_INSTS_VALU_FMA_F64": 4,
               "SQ_INSTS_VALU_INT64": 4, "SQ_INSTS_VALU_TRANS_F64": 16}
        if all(k in avg for k in cls):
            other = avg["SQ_INSTS_VALU"] - sum(avg[k] for k in cls)
            res["valu_issue_cycles_measured"] = sum(avg[k] * c for k, c in cls.items()) + 2 * max(0.0, other)
            res["valu_other_insts"] = other
            res["valu_issue_frac_measured"] = res["valu_issue_cycles_measured"] / res["simd_cycles"]
        res["valu_issue_frac"] = res.get("valu_issue_frac_measured", res["valu_issue_frac_model"])
        res["valu_issue_basis"] = ("per-class costs measured by tools/valu_rate.hip" if "valu_issue_frac_measured" in res
                                   else "model: 2 cycles per wave64 instruction, 4 per f64")
    if "SQ_ACTIVE_INST_VALU2" in avg and "SQ_ACTIVE_INST_VALU" in avg and "SQ_BUSY_CYCLES" in avg:
        # counter-based, no cost model: SQ_ACTIVE_INST_VALU = quad-cycles each wave issues VALU work
        # (summed over waves; 1 per instruction, 2 / 4 for f32 / f64 transcendentals),
        # SQ_ACTIVE_INST_VALU2 = quad-cycles in which two waves' VALU instructions issued together
        # (gfx950 dual issue, counted under both waves above): the SIMD's VALU issue port is busy
        # 4 x (VALU - VALU2) of its cycles
        simd = 32 * avg["SQ_BUSY_CYCLES"]
        res["simd_cycles"] = simd
        res["valu_busy_quads"] = avg["SQ_ACTIVE_INST_VALU"] - avg["SQ_ACTIVE_INST_VALU2"]
        res["valu_busy_frac"] = 4 * res["valu_busy_quads"] / simd
        res["valu_dual_issue_share"] = 2 * avg["SQ_ACTIVE_INST_VALU2"] / avg["SQ_ACTIVE_INST_VALU"]
        for k in ("SCA", "LDS", "MISC", "VMEM"):
            if f"SQ_ACTIVE_INST_{k}" in avg:
                res[f"{k.lower()}_busy_frac"] = 4 * avg[f"SQ_ACTIVE_INST_{k}"] / simd
        if "valu_issue_frac" in res:
            res["valu_issue_frac_class_model"] = res["valu_issue_frac"]
        res["valu_issue_frac"] = res["valu_busy_frac"]
        res["valu_issue_basis"] = ("counters: 4 x (SQ_ACTIVE_INST_VALU - SQ_ACTIVE_INST_VALU2) / (32 x SQ_BUSY_CYCLES), "
                                   "the SIMDs' VALU issue quad-cycles net of dual issue")
    if "GRBM_GUI_ACTIVE" in avg:
        res["simd_cycles_from_grbm"] = 1024 * avg["GRBM_GUI_ACTIVE"] / 8
        if durs:
            res["effective_clock_ghz"] = avg["GRBM_GUI_ACTIVE"] / 8 / res["kernel_ns_under_pmc"]
    if "SQ_THREAD_CYCLES_VALU" in avg and "SQ_ACTIVE_INST_VALU" in avg:
        res["valu_lane_utilization"] = avg["SQ_THREAD_CYCLES_VALU"] / (64 * avg["SQ_ACTIVE_INST_VALU"])
    if "SQ_WAVE_CYCLES" in avg and "simd_cycles" in res:
        # resident waves per SIMD, averaged over the kernel (SQ_WAVE_CYCLES counts quad-cycles);
        # a block that no longer fits in LDS shows here as one wave fewer
        res["avg_waves_per_simd"] = 4 * avg["SQ_WAVE_CYCLES"] / res["simd_cycles"]
    if "SQ_WAVE_CYCLES" in avg:
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if k in avg:
                res[k.lower() + "_share"] = avg[k] / avg["SQ_WAVE_CYCLES"]
    out.write_text(json.dumps(res, indent=1) + "\n")
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
