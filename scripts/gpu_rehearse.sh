#!/bin/bash
# Multi-rank rehearsal of bench.py on a 1-GPU box: 2 ranks share cuda:0,
# collectives over gloo (host).  Then the default N=1 bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/reh
for cfg in "2" "3" "5" "6" "4 --grid4 32"; do
  tag=$(echo $cfg | cut -d' ' -f1)
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 5 --warmup 1 --backend gloo --config $cfg > gpurun_out/reh/n2_cfg$tag.json 2> gpurun_out/reh/n2_cfg$tag.err || { echo "rehearsal cfg$tag failed"; tail -20 gpurun_out/reh/n2_cfg$tag.err; exit 1; }
  echo "cfg$tag:"; cat gpurun_out/reh/n2_cfg$tag.json | cut -c1-400
done
timeout -k 10 240 python bench.py --no-cpu-baseline > gpurun_out/reh/n1.json 2> gpurun_out/reh/n1.err || { echo "n1 failed"; tail gpurun_out/reh/n1.err; exit 1; }
cat gpurun_out/reh/n1.json | cut -c1-600
