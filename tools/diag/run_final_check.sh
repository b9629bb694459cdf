# end-of-session check (GPU box, repo root): GPU suite + bench (tools/gpu_tests.sh) + smoke()
set -o pipefail
export TMPDIR=/tmp
bash tools/gpu_tests.sh r2m || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r2m/smoke.log 2>&1 || { tail -20 gpurun_out/r2m/smoke.log; exit 1; }
tail -3 gpurun_out/r2m/smoke.log
