# XCD chunk (blocks per XCD group, GOL_XCD_CHUNK) at the deep passes, one
# process per value, interleaved twice.
cd $GRAFT_REPO_ROOT
for r in 1 2; do
  for c in 4 8 16 32; do
    GOL_XCD_CHUNK=$c GPPS=12 BANDS=0 TAILS="" ROUNDS=2 GENS=60 timeout -k 10 120 python scripts/rank_sweep.py 262144x262144 | sed "s/^/chunk=$c r$r /" || exit 1
    GOL_XCD_CHUNK=$c GPPS=12 BANDS=0 TAILS="" ROUNDS=2 GENS=60 timeout -k 10 120 python scripts/rank_sweep.py 262144x32768 | sed "s/^/chunk=$c r$r /" || exit 1
  done
done
