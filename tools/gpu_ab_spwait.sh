# Self-play leg: engine base/new x OpenMP wait policy x threads, with the cgroup's throttling
# counters (bench selfplay.cgroup_cpu), one GPU session.   bash tools/gpu_ab_spwait.sh <tag>
set -e
tag=${1:-ab_spwait}
mkdir -p gpurun_out/$tag
cat /sys/fs/cgroup/cpu.max > gpurun_out/$tag/cpu_max.txt 2>&1 || true
F="--steps 5 --warmup 2 --no-cpu --no-train --no-b1 --no-grid --no-aggregate --no-agg-extra --large-batch 0"
for i in 1 2; do
  for mode in base:16 new:16 new:16p new:14p base:16p; do
    lib=${mode%%:*}; th=${mode##*:}; n=${th%p}
    if [ $lib = base ]; then export AZ_AB_MCTS_LIB=libaz_mcts_base.so; else unset AZ_AB_MCTS_LIB; fi
    if [ "$n" != "$th" ]; then export OMP_WAIT_POLICY=passive; else unset OMP_WAIT_POLICY; fi
    timeout -k 10 200 python -u bench.py $F --sp-threads $n 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); s=d['selfplay']; print(json.dumps({'mode':'$mode','games_per_s':s['games_per_s'],'net_wait_s':s['net_wait_s'],'host_s':s['host_s'],'collect_s':s.get('collect_s'),'launch_s':s.get('launch_s'),'cg':s.get('cgroup_cpu')}))" >> gpurun_out/$tag/ab.jsonl
  done
done
