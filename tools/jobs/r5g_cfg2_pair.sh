O=gpurun_out/r5g; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread -p no:cacheprovider -k "act_round or two_stream or compact_trainer or trainer or cfg2" > $O/tests.log 2>&1 || { echo "tests rc=$?" >> $O/job.log; exit 1; }
for w in "1024 512" "512 256" "2048 512" "3072 512" "1024 256" "1024 1024" "2048 256"; do
  set -- $w
  MS_ACT_FIXED_WAVES=$1 MS_ACT_FIXED_COMMON_WAVES=$2 timeout -k 10 300 python bench.py --config cfg2 --no-cpu-baseline > $O/cfg2_$1_$2.json 2> $O/cfg2_$1_$2.err || exit 1
done
MS_ACT_UNPAIRED=1 timeout -k 10 300 python bench.py --config cfg2 --no-cpu-baseline > $O/cfg2_unpaired.json 2> $O/cfg2_unpaired.err || exit 1
echo done >> $O/job.log
