#!/usr/bin/env bash
# One parameterised GPU job (run through gpurun): the steps named on the command line, in order, each
# under its own time limit, the job ending at the first failing step. Outputs go to gpurun_out/<tag>/.
#
# Usage: bash tools/gpu_job.sh <tag> <step> [<step> ...]
#   gputest             the whole -m gpu suite                         -> gputest.log
#   tests:<k-expr>      the -m gpu tests matching a pytest -k expression -> tests.log
#   smoke               __graft_entry__.smoke()                         -> smoke.log
#   bench[:<args>]      the default bench line (extra args after ':', ',' for spaces) -> bench.json
#   cfgs                the cfg2 / cfg4 / cfg5 bench lines              -> cfg{2,4,5}.json
#   profile             profiles/run_profile.sh (kernel trace + env PMC traffic of the bench)
#   profile_cfg:<cfgs>  tools/profile_cfg.sh for the listed configs (',' separated)
#   pmc[:<cfg>:<filter>] profiles/run_pmc.sh (PMC passes of the kernels matching filter)
#   trace5              tools/trace_cfg5.sh (cfg5 frame breakdown)
#   phase               tools/env_phase_probe.py (per-wave phase cycles of the env round)
#   ab:<variant>:<n>[:<args>]  n alternating cfg3 bench lines of tools/_variants/<variant> and the
#                       in-tree library (same box)                   -> ab_<variant>_{base,new}<i>.json
#   waves:<off>:<acc>   cfg3 bench line with the paired act's wave split -> waves_<off>_<acc>.json
#   envab:<VAR=v[+VAR=v]>:<n>[:<args>]  n alternating bench lines with those environment variables and without
#                       (same box; args after ':', ',' for spaces)  -> envab_<vars>_<i>_{with,without}.json
#                       (the one-off A/B jobs of rounds 4-5, e.g. MS_UPDATE_STREAMS=1 at cfg4:
#                        envab:MS_UPDATE_STREAMS=1:2:--config,cfg4,--steps,3,--no-cpu-baseline)
# Example: bash tools/gpu_job.sh r5b gputest smoke bench cfgs profile
set -uo pipefail
TAG="$1"; shift
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp

fail() { echo "step '$1' failed (rc $2)" | tee -a "$O/job.log"; exit "$2"; }

for step in "$@"; do
  IFS=: read -r name a1 a2 a3 <<< "$step"
  echo "$(date +%T) step $step" >> "$O/job.log"
  case "$name" in
    gputest)
      timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider \
        > "$O/gputest.log" 2>&1 || fail "$step" $? ;;
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -v -rP --timeout 400 --timeout-method thread \
        -p no:cacheprovider -k "$a1" > "$O/tests.log" 2>&1 || fail "$step" $? ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || fail "$step" $? ;;
    bench)
      timeout -k 10 400 python bench.py ${a1//,/ } > "$O/bench.json" 2> "$O/bench.err" || fail "$step" $? ;;
    cfgs)
      for c in cfg2 cfg4 cfg5; do
        timeout -k 10 300 python bench.py --config "$c" --no-cpu-baseline > "$O/$c.json" 2> "$O/$c.err" || fail "$step $c" $?
      done ;;
    profile)
      bash profiles/run_profile.sh "$TAG" > "$O/profile.log" 2>&1 || fail "$step" $? ;;
    profile_cfg)
      bash tools/profile_cfg.sh "$TAG" ${a1//,/ } > "$O/profile_cfg.log" 2>&1 || fail "$step" $? ;;
    pmc)
      bash profiles/run_pmc.sh "$TAG" $a1 $a2 > "$O/pmc.log" 2>&1 || fail "$step" $? ;;
    trace5)
      bash tools/trace_cfg5.sh "$TAG" > "$O/trace5.log" 2>&1 || fail "$step" $? ;;
    phase)
      timeout -k 10 300 python tools/env_phase_probe.py > "$O/phase.txt" 2>&1 || fail "$step" $? ;;
    ab)
      B="$R/tools/_variants/$a1/libmarlsched.so"
      [[ -f "$B" ]] || fail "$step (no $B)" 2
      for i in $(seq 1 "${a2:-2}"); do
        MARLSCHED_LENIENT_ABI=1 MARLSCHED_LIB="$B" timeout -k 10 300 python bench.py --no-cpu-baseline --steps 8 ${a3//,/ } \
          > "$O/ab_${a1}_base$i.json" 2> "$O/ab_${a1}_base$i.err" || fail "$step base $i" $?
        timeout -k 10 300 python bench.py --no-cpu-baseline --steps 8 ${a3//,/ } \
          > "$O/ab_${a1}_new$i.json" 2> "$O/ab_${a1}_new$i.err" || fail "$step new $i" $?
      done ;;
    waves)
      MS_ACT_PAIR_WAVES="$a1" MS_ACT_PAIR_COMMON_WAVES="$a2" timeout -k 10 300 python bench.py --no-cpu-baseline \
        --no-step-kernel --steps 6 > "$O/waves_${a1}_${a2}.json" 2> "$O/waves_${a1}_${a2}.err" || fail "$step" $? ;;
    envab)
      n="envab_${a1//[^A-Za-z0-9]/_}"
      for i in $(seq 1 "${a2:-2}"); do
        env ${a1//+/ } timeout -k 10 300 python bench.py ${a3//,/ } > "$O/${n}_${i}_with.json" 2> "$O/${n}_${i}_with.err" \
          || fail "$step with $i" $?
        timeout -k 10 300 python bench.py ${a3//,/ } > "$O/${n}_${i}_without.json" 2> "$O/${n}_${i}_without.err" \
          || fail "$step without $i" $?
      done ;;
    *)
      fail "$step (unknown step)" 2 ;;
  esac
done
echo "$(date +%T) done" >> "$O/job.log"
echo done > "$O/done"
