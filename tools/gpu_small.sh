OUT=gpurun_out/small1
mkdir -p $OUT
for p in 125 250 500; do
timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --paths $p --no-cpu-baseline --no-e2e > $OUT/bench_$p.json 2> $OUT/bench_$p.err || { echo "bench $p failed"; tail $OUT/bench_$p.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench_$p.json'));print($p, d['ms_per_step'], d['value'])"
done
cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --paths 125 --no-cpu-baseline --no-e2e > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1; echo "prof rc=$?"; cd $GRAFT_REPO_ROOT && python tools/prof_summary.py $OUT/prof | head -25
