# Rehearsal of bench.py's N > 1 path on a one-GPU box (2 ranks on cuda:0, gloo collectives):
# independent env blocks, then the shared policy. Timings are meaningless; this checks the code
# path (rank setup, seeds, broadcast, bucket all-reduce, max-over-ranks, rank-0 JSON line).
set -e -o pipefail
cd "$GRAFT_REPO_ROOT"
export NAV_DIST_REHEARSAL=1
OUT=${1:-gpurun_out/dist_rehearsal.log}
ARGS="--gpus 2 --steps 20 --warmup 2 --long-steps 0"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py $ARGS > "$OUT" 2>&1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29532 bench.py $ARGS --shared-policy >> "$OUT" 2>&1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py $ARGS --shared-policy --overlap-collect >> "$OUT" 2>&1
