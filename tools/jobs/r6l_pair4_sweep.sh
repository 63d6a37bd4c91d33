# wave split of cfg4's paired act launch
O=gpurun_out/r6l; mkdir -p $O
for w in ${SWEEP:-"2048 1024" "2048 512" "2048 2048" "1024 1024" "4096 1024" "3072 1536"}; do
  set -- $w
  MS_ACT_PAIR4_WAVES=$1 MS_ACT_PAIR4_COMMON_WAVES=$2 timeout -k 10 300 python bench.py --config cfg4 --steps 3 --no-cpu-baseline > $O/w_$1_$2.json 2>> $O/err.log || exit 1
done
