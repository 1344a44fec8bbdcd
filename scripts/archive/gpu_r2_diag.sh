# Where does time go outside the kernels (hashed / unhashed, 262144^2 and
# 65536^2 at the bench's generation counts)?
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python scripts/hash_wall.py 262144 262144 20 > gpurun_out/r2_hash_wall_262144.log 2>&1
rc=$?; echo "262144 rc=$rc"; cat gpurun_out/r2_hash_wall_262144.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/hash_wall.py 65536 65536 102 > gpurun_out/r2_hash_wall_65536.log 2>&1
rc=$?; echo "65536 rc=$rc"; cat gpurun_out/r2_hash_wall_65536.log; exit $rc
