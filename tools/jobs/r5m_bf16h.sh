# the offer gradient's 16-wide layers on three-term bf16 (MS_GRAD_BF16H=1 variant) vs f32
O=gpurun_out/r5m; mkdir -p $O; export TMPDIR=/tmp
V=$PWD/tools/_variants/bf16h/libmarlsched.so
MARLSCHED_LIB=$V timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "fused_grad or grad_matches" > $O/tests_bf16h.log 2>&1; echo "tests rc=$?" >> $O/job.log
bash tools/gpu_job.sh r5m ab:bf16h:3 || exit 1
for v in base bf16h; do
  if [[ $v == base ]]; then unset MARLSCHED_LIB; else export MARLSCHED_LIB=$V; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/prof_$v.log 2>&1 || exit 1
done
echo done >> $O/job.log
