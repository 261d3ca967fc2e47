set -o pipefail
mkdir -p gpurun_out
for g in 0 1; do
timeout -k 10 300 python bench.py --model inception_v3_slim_old --steps 20 --warmup 5 --graph $g > gpurun_out/bi_$g.log 2>&1 || { tail -20 gpurun_out/bi_$g.log; exit 1; }
echo "graph=$g $(tail -1 gpurun_out/bi_$g.log | cut -c1-200)"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --graph $g > gpurun_out/br_$g.log 2>&1 || { tail -20 gpurun_out/br_$g.log; exit 1; }
echo "graph=$g $(tail -1 gpurun_out/br_$g.log | cut -c1-200)"
done
