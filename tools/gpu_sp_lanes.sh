mkdir -p gpurun_out/spl
for L in 2 3 4; do
  timeout -k 10 300 python -u bench.py --no-cpu --no-grid --no-b1 --no-train --large-batch 0 --no-aggregate --steps 5 --warmup 2 --sp-lanes $L > gpurun_out/spl/b$L.json 2> gpurun_out/spl/b$L.err || exit 1
done
