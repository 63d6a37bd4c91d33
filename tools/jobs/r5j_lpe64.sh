O=gpurun_out/r5j; mkdir -p $O
for i in 1 2; do
  timeout -k 10 300 python bench.py --config cfg2 --no-cpu-baseline > $O/cfg2_fused_$i.json 2> $O/err_$i.log || exit 1
  MS_ENV_MIN_WAVES=4096 timeout -k 10 300 python bench.py --config cfg2 --no-cpu-baseline > $O/cfg2_fused_w4096_$i.json 2>> $O/err_$i.log || exit 1
  MS_ENV_MIN_WAVES=4096 MS_ENV_FUSED_ACT=0 timeout -k 10 300 python bench.py --config cfg2 --no-cpu-baseline > $O/cfg2_plain_w4096_$i.json 2>> $O/err_$i.log || exit 1
done
echo done >> $O/job.log
