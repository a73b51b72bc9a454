# FwFM-only forward at the driver's 20 steps: stream count (3 does not divide 20)
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r03aw}
run() { local name=$1 t=$2; shift 2; timeout -k 10 "$t" "$@" > gpurun_out/${T}_$name.log 2>&1; local rc=$?; echo "$name rc=$rc: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/${T}_$name.log) $(grep -o '"streams_in_region": {[^}]*}' gpurun_out/${T}_$name.log)"; [ $rc -ge 124 ] && exit $rc; return $rc; }
for s in 3 2 4 5; do
  run fwfm20_s$s 200 python bench.py --config fwfm --steps 20 --warmup 5 --no-cpu-baseline --streams $s || exit 1
done
for s in 3 4 5; do
  run fwfm2000_s$s 200 python bench.py --config fwfm --steps 2000 --warmup 400 --no-cpu-baseline --streams $s || exit 1
done
run fwfm20_s3b 200 python bench.py --config fwfm --steps 20 --warmup 5 --no-cpu-baseline --streams 3 || exit 1
run fwfm20_s4b 200 python bench.py --config fwfm --steps 20 --warmup 5 --no-cpu-baseline --streams 4 || exit 1
echo done
