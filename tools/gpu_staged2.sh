# 2-rank rehearsal of bench.py's N>1 path on one GPU (gloo-staged exchange; never a reported number)
set -o pipefail
mkdir -p gpurun_out
DR_BENCH_GLOO_STAGED=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 3 --rows 3000000 --cpu-seconds 0 --train-steps 0 --no-deepfm > gpurun_out/staged2.log 2>&1
rc=$?; grep -E "engine|lookup kernel|^\{" gpurun_out/staged2.log | cut -c1-400; exit $rc
