# returns staged too (last row trimmed to the window): keyed / trainer tests incl. the cfg3 E=16384 case, then cfg3/cfg4 benches
O=gpurun_out/r6t; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "keyed or compact_trainer or fullsize" > $O/tests.log 2>&1 || { echo "tests rc=$?" >> $O/job.log; exit 1; }
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 1 --no-step-kernel --no-cpu-baseline > $O/cfg3_$i.json 2>> $O/err.log || exit 1
  MS_KEY_GATHER_ROWS=0 timeout -k 10 300 python bench.py --steps 20 --warmup 1 --no-step-kernel --no-cpu-baseline > $O/cfg3_lane_$i.json 2>> $O/err.log || exit 1
done
