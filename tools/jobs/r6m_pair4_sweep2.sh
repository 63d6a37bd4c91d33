# second pass over the best wave splits of cfg4's paired act launch
O=gpurun_out/r6m; mkdir -p $O
for w in "3072 1536" "1024 1024" "1536 1536" "1024 512" "3072 1536" "1024 1024" "1536 768"; do
  set -- $w
  MS_ACT_PAIR4_WAVES=$1 MS_ACT_PAIR4_COMMON_WAVES=$2 timeout -k 10 300 python bench.py --config cfg4 --steps 3 --no-cpu-baseline > $O/w_$1_$2_$RANDOM.json 2>> $O/err.log || exit 1
done
