# dynamic-admission bench: plain and under torchrun (1 rank, RCCL all-gather) (gpurun helper)
set -e
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --workload dynamic --no-cpu-baseline > gpurun_out/dyn.json 2> gpurun_out/dyn.err
tail -1 gpurun_out/dyn.json
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --workload dynamic --no-cpu-baseline --streams 64 > gpurun_out/dyn_tr.json 2> gpurun_out/dyn_tr.err
tail -1 gpurun_out/dyn_tr.json
