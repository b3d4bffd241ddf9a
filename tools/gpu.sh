#!/bin/bash
# One parametrised driver for GPU-box evidence runs (replaces the one-off
# gpu_rNN*.sh wrappers). Run on the box via gpurun, from the repo root:
#   bash tools/gpu.sh <recipe> [<recipe> ...]
# Recipes run in order; the first failure (non-zero, timeout, fault) ends the
# call. Each step has its own time limit; logs land in gpurun_out/<name>.log.
#   tests[:<pytest -k expr>]  GPU test suite (or a -k subset)
#   testfile:<path>           one test file
#   smoke                     __graft_entry__.smoke()
#   bench[:<args>]            python bench.py <args> (commas -> spaces)
#   prof                      kernel trace + stats of the default bench (no cpu baseline)
#   pmc                       round PMC passes (tools/gpu_round_pmc.sh), OGS_COMMIT=<sha>
#   c2scale[:<args>]          C2 kernel time vs batch size in one process (tools/c2_scaling.py)
#   sq:<tag>:<bench args>     one SQ counter pass (wave-cycle split, LDS conflicts) over
#                             `python3 bench.py <bench args>` (commas -> spaces)
#   sqlds:<tag>:<bench args>  second SQ pass: LDS instruction / wait counters
#   stamps:<as-rank>          LDS SPF phase stamps (make stamps; tools/c3_stamps.py --lds)
#   timeline:<as-rank>[:o=v+..] C3 one-launch item timeline (tools/c3_timeline.py)
#   ab:<as-rank>:<A>:<B>[:..] in-process C3 option A/B (tools/c3_opt_ab.py), variants
#                             are name=value lists joined by '+'
#   benchab:<config>:<A>:<B>[:..] any bench.py config, variants interleaved twice, each
#                             a '+'-joined list of engine options name=value (--opt),
#                             bench flags --name=value written name=value with a
#                             leading '-' (e.g. -c5-streams=2), or lib=base
#                             (openr_amd/lib/libopenr_gpu_base.so, tools/build_ab_base.sh)
#                             or tree=<dir> (another built tree's bench.py, e.g. ab/r04:
#                             a git worktree of an older commit, built, copied in)
#                             or an OGS_* environment variable (OGS_SLOT_BANKS=0)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp && cd "$GRAFT_REPO_ROOT" || exit 1
COMMIT=${OGS_COMMIT:-unknown}

step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name: $*"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; grep -v amdgpu.ids "gpurun_out/$name.log" | tail -4 | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
}

SQ1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU"
SQ2="SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_INSTS_SALU SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES"

n=0
for recipe in "$@"; do
  n=$((n + 1))
  kind=${recipe%%:*}
  rest=${recipe#*:}
  [ "$rest" = "$recipe" ] && rest=""
  case $kind in
    tests)
      if [ -n "$rest" ]; then
        step "pytest_$n" 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider -x --timeout 200 --timeout-method thread -k "$rest"
      else
        step pytest_gpu 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider -x --timeout 200 --timeout-method thread
      fi ;;
    testfile)
      step "pytest_$n" 300 python -u -m pytest "$rest" -v -p no:cacheprovider -x --timeout 200 --timeout-method thread ;;
    smoke)
      step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)
      step "bench_$n" 900 python bench.py ${rest//,/ } ;;
    prof)
      step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- python3 bench.py --no-cpu-baseline --no-extras
      grep -v "at::native" gpurun_out/prof/bench_kernel_stats.csv | cut -c1-200 | head -20 ;;
    pmc)
      OGS_COMMIT=$COMMIT step pmc 900 bash tools/gpu_round_pmc.sh ;;
    sq|sqlds)
      tag=${rest%%:*}; args=${rest#*:}
      C=$SQ1; [ "$kind" = sqlds ] && C=$SQ2
      # a counter pass that cannot be collected may hang past SIGTERM: KILL
      echo "=== ${kind}_$tag"
      mkdir -p "gpurun_out/${kind}_$tag" && echo "$COMMIT" > "gpurun_out/${kind}_$tag/commit.txt"
      timeout -s KILL 150 rocprofv3 --pmc $C --output-format csv -d "gpurun_out/${kind}_$tag" -o sq -- python3 bench.py ${args//,/ } > "gpurun_out/${kind}_$tag.log" 2>&1
      rc=$?; echo "=== ${kind}_$tag rc=$rc"; tail -3 "gpurun_out/${kind}_$tag.log" | cut -c1-300
      [ $rc -eq 0 ] || exit $rc ;;
    stamps)
      OGS_LIB=openr_amd/lib/libopenr_gpu_stamps.so step "stamps_$n" 300 python -u tools/c3_stamps.py --lds --as-rank "$rest" --opt route_stream=4 ;;
    timeline)
      OGS_LIB=openr_amd/lib/libopenr_gpu_stamps.so step "timeline_$n" 300 python -u tools/c3_timeline.py --as-rank "${rest%%:*}" $(for o in $(echo "${rest#*:}" | tr '+' ' '); do [ "$o" != "${rest%%:*}" ] && echo "--opt $o"; done) ;;
    ab)
      IFS=: read -r -a parts <<< "$rest"
      rank=${parts[0]}; vs=()
      for v in "${parts[@]:1}"; do vs+=("${v//+/,}"); done
      step "ab_$n" 600 python -u tools/c3_opt_ab.py --pairs 4 --as-rank "$rank" "${vs[@]}"
      grep '^{' "gpurun_out/ab_$n.log" | cut -c1-200 ;;
    benchab)
      IFS=: read -r -a parts <<< "$rest"
      cfg=${parts[0]}
      for rep in 1 2; do
        vi=0
        for v in "${parts[@]:1}"; do
          vi=$((vi + 1)); args=(); lib=""; envs=(); tree=.
          for kv in ${v//+/ }; do
            case $kv in
              lib=base) lib=openr_amd/lib/libopenr_gpu_base.so ;;
              tree=*) tree=${kv#tree=} ;;
              OGS_*=*) envs+=("$kv") ;;
              -*) args+=("-${kv%%=*}" "${kv#*=}") ;;
              *) args+=(--opt "$kv") ;;
            esac
          done
          log="gpurun_out/benchab_${n}_${cfg}_${vi}_$rep.log"
          env "${envs[@]}" OGS_LIB=$lib timeout -k 10 300 python3 "$tree/bench.py" --config "$cfg" --steps 10 --warmup 2 \
            --no-cpu-baseline "${args[@]}" > "$log" 2>&1
          rc=$?; [ $rc -eq 0 ] || { tail -5 "$log"; exit $rc; }
          echo "$cfg [$v] rep $rep: $(grep '^{' "$log" | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["unit"], d["ms_per_step"], "ms", {k: v for k, v in d.items() if k.endswith("digest") or k == "golden"})')"
        done
      done ;;
    c2scale)
      step "c2scale_$n" 300 python -u tools/c2_scaling.py ${rest//,/ } ;;
    *)
      echo "unknown recipe $recipe"; exit 2 ;;
  esac
done
echo "=== all done"
