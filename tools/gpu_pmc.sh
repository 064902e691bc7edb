#!/bin/bash
# PMC passes of one bench workload: one rocprofv3 --pmc run per counter group (no --pmc mixed with
# tracing options; at most 8 SQ / 4 TCC / 2 GRBM per pass), each under its own time limit, then
# tools/pmc_summary.py -> <outdir>/summary.json.
#   tools/gpu_pmc.sh <outdir under gpurun_out> [bench.py args]   (PASSES="3 6": those passes only)
# Counters absent from `rocprofv3 -L` on this box are dropped from their pass.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/$1
shift
ARGS="--steps 1 --warmup 0 --no-cpu-baseline $*"
mkdir -p "$OUT"
# counters are only collected on a library built from committed sources: its build stamp
# (crt_build_info: source sha + git commit, Makefile) must not be dirty, and its source sha must be
# that of the sources in this tree (the .so was built from them)
(cd "$R" && python -c "
import hashlib, subprocess, sys
from bench import build_stamp
st = build_stamp()
srcs = subprocess.run(['make', '-s', '-C', 'cpp_raytracer_amd', 'stamp-srcs'], capture_output=True,
                      text=True, check=True).stdout.split()
h = hashlib.sha256(b''.join(open('cpp_raytracer_amd/' + f, 'rb').read() for f in srcs)).hexdigest()[:16]
ok = not st['git_dirty'] and st['source_sha'] == h
print(('pmc: library ' if ok else 'pmc: REFUSED, library ') + st['build_info'] + ' tree src=' + h)
sys.exit(0 if ok else 3)") || exit 3
export TMPDIR=/tmp
cd /tmp
[ -s "$R/gpurun_out/counters_list.txt" ] || timeout -k 10 120 rocprofv3 -L > "$R/gpurun_out/counters_list.txt" 2>&1
have() { grep -qw "$1" "$R/gpurun_out/counters_list.txt"; }
pick() { local out=""; for c in "$@"; do have "${c%_sum}" && out="$out $c"; done; echo $out; }
P1=$(pick FETCH_SIZE GRBM_GUI_ACTIVE)
P2=$(pick WRITE_SIZE TCC_HIT_sum TCC_MISS_sum)
P3=$(pick SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU)
P4=$(pick SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_LDS_BANK_CONFLICT)
P5=$(pick SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU)
# issue slots: VALU quad-cycles per wave, the quad-cycles two VALU instructions issued together
# (gfx950 dual issue), and the other issue units
P6=$(pick SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_BUSY_CYCLES SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE)
i=0
for grp in "$P1" "$P2" "$P3" "$P4" "$P5" "$P6"; do
  i=$((i+1))
  [ -n "$grp" ] || continue
  case " ${PASSES:-1 2 3 4 5 6} " in *" $i "*) ;; *) continue ;; esac
  timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$OUT/p$i" -o run -- python3 "$R/bench.py" $ARGS > "$OUT/bench_p$i.json" 2> "$OUT/bench_p$i.err" || { echo "pmc pass $i ($grp) failed"; tail -5 "$OUT/bench_p$i.err"; exit 1; }
  echo "pmc pass $i ok: $grp"
done
cd "$R" && python tools/pmc_summary.py "$OUT" "$OUT/summary.json" > /dev/null && echo "pmc summary ok: $OUT/summary.json"
