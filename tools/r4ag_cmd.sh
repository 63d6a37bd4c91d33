# act_pair offer wave count around the default (cfg3, one box, alternating)
set -o pipefail
O=gpurun_out/r4ag
mkdir -p $O
for rep in 1 2; do
  for wv in 2048 1792 2304 2560 4096; do
    MS_ACT_PAIR_WAVES=$wv timeout -k 10 300 python bench.py --no-cpu-baseline --no-step-kernel --steps 6 > $O/w_${wv}_$rep.json 2> $O/w_${wv}_$rep.err || exit 1
  done
done
echo done > $O/done
