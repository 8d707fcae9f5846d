# Round 4: the full GPU suite, smoke and the repeated full-size C2 parity check (debug_mb_race).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_all.log 2>&1 || { tail -40 gpurun_out/pytest_all.log; exit 1; }
tail -3 gpurun_out/pytest_all.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python -u tools/debug_mb_race.py 3 > gpurun_out/race_final.log 2>&1 || { tail -20 gpurun_out/race_final.log; exit 1; }
grep "== rep" gpurun_out/race_final.log
