#!/bin/bash
# One parametrised recipe for every GPU-box measurement (run through gpurun).  Each
# step writes under gpurun_out/; chain steps with && so the first failure ends the call.
#
#   bash tools/recipe.sh suite    <tag>                        full `pytest -m gpu`
#   bash tools/recipe.sh tests    <tag> [LIB=<.so>] <pytest args...>   a subset (optionally on a variant library)
#   bash tools/recipe.sh bench    <tag> [bench args...]        bench.py line -> <tag>_bench.json (+ .err)
#   bash tools/recipe.sh evidence <tag>                        PMC traffic per shape, rocprofv3 stats of the
#                                                              1080p and 4K training legs, default bench line
#   bash tools/recipe.sh layers   <tag> <layers> <ops> <lib.so>...   per-layer A/B: in-tree library vs variants,
#                                                              interleaved twice (tools/bench_layers.py)
#   bash tools/recipe.sh env      <tag> "<VAR=value>" <layers> <ops>  per-layer A/B under an environment switch
#   bash tools/recipe.sh benchab  <tag> "<VAR=value>|<lib.so>" [bench args...]   bench A/B, interleaved twice
#                                                              (BASE=<lib.so>: another baseline than the in-tree one)
#   bash tools/recipe.sh pmc      <tag> <layers> <ops> "<counters>"  one rocprofv3 --pmc pass over bench_layers
#   bash tools/recipe.sh isolate  <tag> <test file> "<-k expr>" "<VAR=value>"...   one test under each switch
#                                                              (baseline first); a test failure does not end the
#                                                              call, a timeout / crash does
#   bash tools/recipe.sh benchattrib <tag> <lib.so|""> [bench args...]  tools/pmc_attrib.sh's four counter passes over
#                                                              one warmup + one timed + one instrumented training step
#                                                              (post-process: python tools/pmc_attrib.py
#                                                              gpurun_out/attrib_<tag> --steps 3)
#   bash tools/recipe.sh mfma     <tag> [bench args...]        MFMA-busy + GRBM_GUI_ACTIVE pass over one bench step
#                                                              (post-process: python tools/mfma_busy.py <csv>)
#
# Variant libraries come from tools/build_variant.sh (CPU side, before the call).
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out
LIB=$R/cnn_itmo_amd/lib/libcnnitmo.so
T="timeout -k 10"
cmd=$1; tag=$2; shift 2
mkdir -p "$O"
cd "$R"

layers() {  # lib layers ops
  CNNITMO_LIB=$1 $T 180 python "$R/tools/bench_layers.py" --layers "$2" --ops "$3" --iters 5 2>&1 | grep -v amdgpu.ids
}

case $cmd in
suite)
  $T 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/${tag}_gpu_tests.log" 2>&1
  tail -2 "$O/${tag}_gpu_tests.log" ;;
tests)
  lib=$LIB
  case $1 in LIB=*) lib=${1#LIB=}; shift ;; esac
  CNNITMO_LIB=$lib $T 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread "$@" > "$O/${tag}_tests.log" 2>&1
  tail -2 "$O/${tag}_tests.log" ;;
bench)
  $T 900 python3 bench.py "$@" > "$O/${tag}_bench.json" 2> "$O/${tag}_bench.err"
  cat "$O/${tag}_bench.json" ;;
evidence)
  bash "$R/tools/pmc_traffic.sh"
  bash "$R/tools/profile_round.sh" "$tag" --steps 5 --warmup 2 --infer-batch 0 --ns-batch 0 --k4-batch 0 --f32-train-batch 0
  bash "$R/tools/profile_round.sh" "${tag}_4k" --height 2160 --width 3840 --batch 8 --steps 5 --warmup 2 \
    --infer-batch 0 --ns-batch 0 --k4-batch 0 --f32-train-batch 0
  cd "$R"
  $T 900 python3 bench.py > "$O/${tag}_bench.json" 2> "$O/${tag}_bench.err"
  cat "$O/${tag}_bench.json" ;;
layers)
  L=$1; P=$2; shift 2
  for rep in 1 2; do
    for lib in "$LIB" "$@"; do echo "== $(basename "$lib")"; layers "$lib" "$L" "$P"; done
  done > "$O/${tag}_ab.txt" 2>&1
  cat "$O/${tag}_ab.txt" ;;
env)
  sw=$1; L=$2; P=$3
  for e in "" "$sw" "" "$sw"; do
    echo "== ${e:-baseline}"
    env $e CNNITMO_LIB=$LIB $T 180 python "$R/tools/bench_layers.py" --layers "$L" --ops "$P" --iters 5 2>&1 | grep -v amdgpu.ids
  done > "$O/${tag}_ab.txt" 2>&1
  cat "$O/${tag}_ab.txt" ;;
benchab)
  sw=$1; shift
  for e in "" "$sw" "" "$sw"; do
    case $e in *.so) envs="CNNITMO_LIB=$e" ;; "") envs="CNNITMO_LIB=${BASE:-$LIB}" ;; *) envs=$e ;; esac
    echo "== ${e:-baseline}"
    env $envs $T 600 python3 bench.py --no-cpu "$@" 2>> "$O/${tag}_ab.err" | grep -E '^\{' | python3 -c \
      "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], d['ms_per_step'], r['kernel'], r['achieved'])"
  done > "$O/${tag}_ab.txt"
  cat "$O/${tag}_ab.txt" ;;
pmc)
  L=$1; P=$2; ctr=$3
  cd /tmp && export TMPDIR=/tmp
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d "$O/pmc_$tag" -o run -- \
    python3 "$R/tools/bench_layers.py" --layers "$L" --ops "$P" --iters 1 > "$O/pmc_${tag}.log" 2>&1 ;;
isolate)
  f=$1; k=$2; shift 2
  for e in "" "$@"; do
    env $e timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread "$f" -k "$k" \
      > "$O/${tag}_iso.log.tmp" 2>&1 && rc=0 || rc=$?
    echo "== ${e:-baseline} rc=$rc: $(tail -1 "$O/${tag}_iso.log.tmp")"
    cat "$O/${tag}_iso.log.tmp" >> "$O/${tag}_iso.log"
    [ $rc -le 1 ] || exit $rc
  done | tee "$O/${tag}_iso.txt"
  rm -f "$O/${tag}_iso.log.tmp" ;;
benchattrib)
  lib=${1:-$LIB}; shift
  case $lib in /*) ;; *) lib=$R/$lib ;; esac
  A=$O/attrib_$tag
  mkdir -p "$A"
  cd /tmp && export TMPDIR=/tmp
  i=0
  for ctr in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_VALU_MFMA_COEXEC_CYCLES GRBM_GUI_ACTIVE" \
             "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_SALU SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE" \
             "SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVES GRBM_GUI_ACTIVE" \
             "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INST_LEVEL_LDS SQ_INST_LEVEL_VMEM SQ_LDS_UNALIGNED_STALL SQ_INST_CYCLES_VMEM_WR GRBM_GUI_ACTIVE"; do
    CNNITMO_LIB=$lib timeout -s KILL 240 rocprofv3 --pmc $ctr --output-format csv -d "$A/p$i" -o run -- \
      python3 "$R/bench.py" --no-cpu --steps 1 --warmup 1 --infer-batch 0 --ns-batch 0 --k4-batch 0 \
      --f32-train-batch 0 "$@" > "$A/p$i.log" 2>&1
    i=$((i+1))
  done
  echo "benchattrib $tag: $i passes" ;;
mfma)
  cd /tmp && export TMPDIR=/tmp
  timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
    --output-format csv -d "$O/mfma_$tag" -o run -- python3 "$R/bench.py" --no-cpu --steps 1 --warmup 1 \
    --infer-batch 0 --ns-batch 0 --k4-batch 0 --f32-train-batch 0 "$@" > "$O/mfma_${tag}.log" 2>&1 ;;
*)
  echo "unknown recipe step: $cmd" >&2; exit 2 ;;
esac
