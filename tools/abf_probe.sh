# A/B of an env switch on the BCE bench line (dev).  usage: bash tools/abf_probe.sh VAR "v1 v2 ..."
cd ${GRAFT_REPO_ROOT:-/root/repo}; mkdir -p gpurun_out/abf
for v in $2; do
  export $1=$v
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-recommend > gpurun_out/abf/b$v.log 2>&1 || exit 1
  tail -1 gpurun_out/abf/b$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1=$v', round(d['ms_per_step']*1e3,1), 'us/step', {k: round(v,1) for k,v in (d['kernel_us'] or {}).items()})"
done
