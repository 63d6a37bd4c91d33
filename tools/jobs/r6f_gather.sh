# row-staged key gather: keyed-gradient / trainer tests, then A/B (MS_KEY_GATHER_ROWS=0: per-lane gather) at cfg3 and cfg4
O=gpurun_out/r6f; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "key or fused_grad or fullsize or union or trainer" > $O/tests.log 2>&1 || { echo "tests rc=$?" >> $O/job.log; exit 1; }
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 1 --no-step-kernel --no-cpu-baseline > $O/cfg3_rows_$i.json 2> $O/err.log || exit 1
  MS_KEY_GATHER_ROWS=0 timeout -k 10 300 python bench.py --steps 20 --warmup 1 --no-step-kernel --no-cpu-baseline > $O/cfg3_lane_$i.json 2>> $O/err.log || exit 1
  timeout -k 10 300 python bench.py --config cfg4 --steps 3 --no-cpu-baseline > $O/cfg4_rows_$i.json 2>> $O/err.log || exit 1
  MS_KEY_GATHER_ROWS=0 timeout -k 10 300 python bench.py --config cfg4 --steps 3 --no-cpu-baseline > $O/cfg4_lane_$i.json 2>> $O/err.log || exit 1
done
