# round-4 A/B (via gpurun): new-kernel GPU tests, then cfg3 / cfg4 / cfg5 bench lines of the previous
# library (tools/_variants/base, round-3 HEAD) against the in-tree one
set -eo pipefail
O=gpurun_out/r4c
mkdir -p $O
timeout -k 10 300 python tools/env_phase_probe.py > $O/phase_new.txt 2>&1 || echo "probe failed rc=$?" >> $O/phase_new.txt
B=$PWD/tools/_variants/base/libmarlsched.so
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "many_groups or hip_update or hip_graph or capture or kat or codec or env_gpu" > $O/tests_new.log 2>&1 || echo "tests failed rc=$?" >> $O/tests_new.log
for i in 1 2; do
  MARLSCHED_LIB=$B timeout -k 10 300 python bench.py --no-cpu-baseline --steps 8 > $O/cfg3_base$i.json 2> $O/cfg3_base$i.err
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 8 > $O/cfg3_new$i.json 2> $O/cfg3_new$i.err
done
MARLSCHED_LIB=$B timeout -k 10 300 python bench.py --config cfg4 --no-cpu-baseline --steps 2 > $O/cfg4_base.json 2> $O/cfg4_base.err
timeout -k 10 300 python bench.py --config cfg4 --no-cpu-baseline --steps 2 > $O/cfg4_new.json 2> $O/cfg4_new.err
timeout -k 10 300 python bench.py --config cfg5 --no-cpu-baseline --steps 1 > $O/cfg5_new.json 2> $O/cfg5_new.err
echo done > $O/done
