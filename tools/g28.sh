# round 6, call 28: the final library's longer records — a 2000-step tail
# probe, config 5 appended (the FMinIter flow), and the full per-rank share
# tables of configs 4 and 5 (T1 and N = 2, 4, 8 shares on this box)
set -o pipefail
O=gpurun_out
step() { local lim=$1 log=$2; shift 2; timeout -k 10 "$lim" "$@" > "$log" 2>&1; local rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; tail -30 "$log"; exit $rc; fi; }
step 400 $O/g28_tail.log python tools/tail_probe.py --steps 2000 --warmup 5 --tag final_g28
tail -3 $O/g28_tail.log
step 600 $O/g28_cfg5app.err python bench.py --config 5 --appending --steps 20 --warmup 2
grep '^{' $O/g28_cfg5app.err > $O/g28_cfg5app.json
python -c "import json; d=json.loads(open('$O/g28_cfg5app.json').read().strip().splitlines()[-1]); print('cfg5 appended', d.get('p50_step_ms'), d['ms_per_step'], d.get('host_phases_us'))"
step 600 $O/g28_cfg5.err python bench.py --config 5 --steps 20 --warmup 2
grep '^{' $O/g28_cfg5.err > $O/g28_cfg5.json
python -c "import json; d=json.loads(open('$O/g28_cfg5.json').read().strip().splitlines()[-1]); print('cfg5 frozen', d.get('p50_step_ms'), d['ms_per_step'], d.get('host_phases_us'))"
step 500 $O/g28_rank5.txt python tools/rank_share.py --config 5 --steps 8 --json $O/g28_rank5.json
grep -v amdgpu $O/g28_rank5.txt
step 500 $O/g28_rank4.txt python tools/rank_share.py --config 4 --steps 10 --json $O/g28_rank4.json
grep -v amdgpu $O/g28_rank4.txt
