# A/B on one box: policy_old sync as one multi-tensor copy (default) vs a copy per tensor
O=gpurun_out/r6e; mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 1 --no-step-kernel --no-cpu-baseline > $O/foreach_$i.json 2> $O/err.log || exit 1
  MS_SYNC_FOREACH=0 timeout -k 10 300 python bench.py --steps 20 --warmup 1 --no-step-kernel --no-cpu-baseline > $O/percopy_$i.json 2>> $O/err.log || exit 1
done
