O=gpurun_out/r5i; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "fused_env_act or compact_trainer or act_round or cfg2" > $O/tests.log 2>&1 || { echo "tests rc=$?" >> $O/job.log; exit 1; }
for i in 1 2; do
  timeout -k 10 300 python bench.py --config cfg2 --no-cpu-baseline > $O/cfg2_fused_$i.json 2> $O/cfg2_fused_$i.err || exit 1
  MS_ENV_FUSED_ACT=0 timeout -k 10 300 python bench.py --config cfg2 --no-cpu-baseline > $O/cfg2_plain_$i.json 2> $O/cfg2_plain_$i.err || exit 1
done
echo done >> $O/job.log
