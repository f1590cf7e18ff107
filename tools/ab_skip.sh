set -e
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $R/gpurun_out/ab1
for i in 1 2; do
for n in base noreduce nopixg nofinal; do
  echo -n "$n: "; (cd $R/ab/$n && timeout -k 10 300 python bench.py --no-cpu-baseline --no-extra-modes --steps 10 --warmup 2 2>/dev/null | grep '^{' | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")
done
done
