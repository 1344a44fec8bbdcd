#!/bin/bash
# Machine scheduler of the step kernels: max-ilp (shipped, in-tree) vs the
# default, iterative-minreg and iterative-maxocc strategies (ab/s_*): the
# driver's command, alternating, two rounds, one box; then one parity pass
# over the full-size tests with the best-looking alternative is left to a
# later call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/r4_sched.ilp$r.json 2> gpurun_out/r4_sched.ilp$r.err || exit 1
  for v in default minreg maxocc; do
    GOL_LIB_PATH=$PWD/ab/s_$v/lib/libgol.so timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/r4_sched.$v$r.json 2> gpurun_out/r4_sched.$v$r.err || exit 1
  done
done
