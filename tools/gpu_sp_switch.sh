# GPU-box: self-play games/s with the lane loop's host settings -- GIL switch interval
# (AZ_SP_SWITCH_INTERVAL: 0.2 ms default, 0 = the interpreter's 5 ms) and the cyclic GC paused
# (default) or running (AZ_SP_GC=1) -- alternating, then the pipeline timeline with the defaults.
#   bash tools/gpu_sp_switch.sh TAG
set -u
cd "$GRAFT_REPO_ROOT"
R=gpurun_out/${1:-sw}; mkdir -p $R
run() {   # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --no-grid --no-train --no-b1 --no-aggregate --large-batch 0 --sp-check 0 > $R/sp_$name.json 2>> $R/err.txt
}
for i in 1 2 3; do
  run new_$i AZ_SP_SWITCH_INTERVAL=0.0002 || exit $?
  run old_$i AZ_SP_SWITCH_INTERVAL=0 AZ_SP_GC=1 || exit $?
done
timeout -k 10 300 python tools/sp_pipeline_probe.py 8192 > $R/pipe.txt 2>> $R/err.txt || exit $?
cp gpurun_out/sp_timeline.json $R/sp_timeline.json
