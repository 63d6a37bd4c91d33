# single-action last tile (kX1) in the PPO gradient: tests, then cfg4 A/B (MS_GRAD_X1=0: on the MFMA)
O=gpurun_out/r6i; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "fused_grad or cfg4 or compact_variants or resynced" > $O/tests.log 2>&1 || { echo "tests rc=$?" >> $O/job.log; exit 1; }
for i in 1 2; do
  timeout -k 10 300 python bench.py --config cfg4 --steps 3 --no-cpu-baseline > $O/cfg4_x1_$i.json 2> $O/err.log || exit 1
  MS_GRAD_X1=0 timeout -k 10 300 python bench.py --config cfg4 --steps 3 --no-cpu-baseline > $O/cfg4_mfma_$i.json 2>> $O/err.log || exit 1
done
