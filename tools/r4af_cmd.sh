# act_pair wave split re-check at the round-4 state (cfg3, one box, alternating)
set -o pipefail
O=gpurun_out/r4af
mkdir -p $O
for rep in 1 2; do
  for cfg in "2048 768" "3072 768" "2048 1536" "1536 768"; do
    set -- $cfg
    MS_ACT_PAIR_WAVES=$1 MS_ACT_PAIR_COMMON_WAVES=$2 timeout -k 10 300 python bench.py --no-cpu-baseline --no-step-kernel --steps 6 > $O/w_${1}_${2}_$rep.json 2> $O/w_${1}_${2}_$rep.err || exit 1
  done
done
echo done > $O/done
