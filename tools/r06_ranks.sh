# round-6 multi-rank rehearsal on one GPU (2 ranks, gloo), then share runs
# of the 8-GPU plan's largest share on the full genome
set -o pipefail
O=${O:-r06w}
mkdir -p gpurun_out/$O
GROM_BENCH_ONE_GPU=1 timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --workdir /tmp/gw2 \
  > gpurun_out/$O/bench_2ranks.json 2> gpurun_out/$O/bench_2ranks.log || { tail -20 gpurun_out/$O/bench_2ranks.log; exit 1; }
cat gpurun_out/$O/bench_2ranks.json | cut -c1-400
S=$(python3 -c "
import bench
from grom_amd.shard import assign_chromosomes
names=[n for n,_ in bench.GRCH38]; L=[l for _,l in bench.GRCH38]
sh=assign_chromosomes(L,8); big=max(sh,key=lambda s: sum(L[i] for i in s))
print(','.join(names[i].lower() for i in big))")
echo "largest share: $S"
OUT=$O tools/session.sh genome 1.0 -- share $S 4
