# Same-box A/B of non-temporal cache hints (ab/<v> built with
# -DGOL_NT_STORES=1 / -DGOL_NT_LOADS=1, scripts/ab_build.sh) vs the in-tree build.
cd $GRAFT_REPO_ROOT
O=gpurun_out/nt
mkdir -p $O
for round in 1 2; do
  for v in cur ntS ntL ntLS; do
    lib=$PWD/akka-game-of-life_amd/lib/libgol.so; [ $v != cur ] && lib=$PWD/ab/$v/lib/libgol.so
    GOL_LIB_PATH=$lib VECS=0 GPPS=1,6 BANDS=0 HASH=0 ROUNDS=2 \
      timeout -k 10 200 python scripts/tune.py 65536 262144 > $O/ab_$v.$round.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "ab $v rc=$rc"; tail -5 $O/ab_$v.$round.log; exit $rc; }
    sed "s/^/$v r$round /" $O/ab_$v.$round.log | cut -c1-118
  done
done
