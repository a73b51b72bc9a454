# deep forward at the driver's 20 steps: stagger of each chip half's second stream
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r03ax}
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > gpurun_out/${T}_$name.log 2>&1; local rc=$?; echo "$name rc=$rc: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/${T}_$name.log) $(grep -o '"streams_in_region": {[^}]*}' gpurun_out/${T}_$name.log)"; [ $rc -ge 124 ] && exit $rc; return $rc; }
for st in 0 5 10 20 40 60 0; do
  run b20_st$st 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --stagger-us $st || exit 1
done
for st in 0 10 40; do
  run b2000_st$st 200 python bench.py --steps 2000 --warmup 400 --no-cpu-baseline --stagger-us $st || exit 1
done
echo done
