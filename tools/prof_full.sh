cd $GRAFT_REPO_ROOT; O=gpurun_out/pf; mkdir -p $O; export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --reg 0.1 --reg-mode full --steps 10 --warmup 3 --no-cpu-baseline --no-recommend > $GRAFT_REPO_ROOT/$O/p.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && python3 tools/prof_collect.py stats $O/prof $O/stats_full.csv
