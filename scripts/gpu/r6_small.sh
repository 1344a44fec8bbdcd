#!/bin/bash
# Round 6: the small-board band rule (gol_schedule.cpp small_board_band):
# parity suites first, then the small-board timings with the library's own
# plan (profiles/r06_small_board_before.txt is the same script on round 5's
# rules), and the driver's bench command (262144^2 and 65536^2 must not move).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
rm -rf gpurun_out/small; mkdir -p gpurun_out/small
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_unhashed_passes.py tests/test_gpu_board_creator.py tests/test_gpu_frontend.py tests/test_gpu_loopback.py > gpurun_out/small/parity.txt 2>&1 || { tail -40 gpurun_out/small/parity.txt; exit 1; }
tail -2 gpurun_out/small/parity.txt
timeout -k 10 200 python3 scripts/small_board.py 1000 > gpurun_out/small/small_board.txt 2>&1 || { cat gpurun_out/small/small_board.txt; exit 1; }
cat gpurun_out/small/small_board.txt
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > gpurun_out/small/bench.json 2> gpurun_out/small/bench.err
rc=$?
python3 -c "import json; d=json.load(open('gpurun_out/small/bench.json')); print(d['value'], d['roofline']['frac'], d['with_state_hash']['value'], d['secondary']['value'], d['parity_ok'])"
exit $rc
