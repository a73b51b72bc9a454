# Round 3: gather floor with 40-B rows vs a packed 64-B-row copy, Criteo tables x1 (MALL) and x8 (HBM)
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-r03ag}
for k in 1 8; do
  for nb in 3 8; do
    timeout -k 10 120 ./tools/ubench_gather $nb $k > gpurun_out/${T}_gather_nb${nb}_k${k}.log 2>&1 || exit $?
    echo "nb=$nb k=$k"; grep -v "^W20" gpurun_out/${T}_gather_nb${nb}_k${k}.log | head -4
  done
done
echo done
