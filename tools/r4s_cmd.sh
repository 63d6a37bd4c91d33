# cfg5 frame breakdown with the idle gaps between dispatches
set -o pipefail
O=gpurun_out/r4s
mkdir -p $O
bash tools/trace_cfg5.sh r4s > $O/trace5.log 2>&1 || exit 1
echo done > $O/done
