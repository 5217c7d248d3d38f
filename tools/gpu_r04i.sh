# self-play engine x wait-policy A/B (cgroup throttle counters); the driver's bench command
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04i
mkdir -p $O
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_args.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json; d=json.loads(open('$O/bench_driver_args.json').read().strip().splitlines()[-1]); print('driver-args bench', d['value'], d['ms_per_step'], d.get('clock_settle'), d['roofline']['frac'], d['selfplay']['games_per_s'], d['selfplay'].get('cgroup_cpu'))"
bash tools/gpu_ab_spwait.sh r04i_spwait || exit 1
cat gpurun_out/r04i_spwait/cpu_max.txt gpurun_out/r04i_spwait/ab.jsonl
echo done > $O/done
