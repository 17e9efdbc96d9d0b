cd $GRAFT_REPO_ROOT
for ev in 1 0; do timeout -k 10 300 python bench.py --no-cpu-baseline --update-events $ev 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print('events',$ev, round(d['value']), 'pivots/s', round(d['ms_per_step']*1000,1),'us/pivot', d['roofline']['avg_launch_us'])" || exit 1; done
timeout -k 10 300 python bench.py --no-cpu-baseline --config config2 --steps 1900 --warmup 50 --update-events 0 2>/dev/null | tail -1 | cut -c1-400
