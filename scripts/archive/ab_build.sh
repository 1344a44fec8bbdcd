#!/bin/bash
# Build libgol.so from another revision of csrc/ (or a patched copy) into
# ab/<name>/lib/libgol.so for same-box A/B timing (GOL_LIB_PATH=...).
#   scripts/ab_build.sh <name> <git-rev | WORKTREE>
set -e
name=$1; rev=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
D=$ROOT/ab/$name
rm -rf "$D"; mkdir -p "$D/pkg" "$D/include" "$D/tmp"
if [ "$rev" = "WORKTREE" ]; then
  (cd "$ROOT" && tar -c akka-game-of-life_amd/csrc akka-game-of-life_amd/Makefile include) | tar -x -C "$D/tmp"
else
  git -C "$ROOT" archive "$rev" akka-game-of-life_amd/csrc akka-game-of-life_amd/Makefile include | tar -x -C "$D/tmp"
fi
mv "$D/tmp/akka-game-of-life_amd"/* "$D/pkg/"; mv "$D/tmp/include"/* "$D/include/"; rm -rf "$D/tmp"
make -C "$D/pkg" -j8 lib/libgol.so EXTRA_HIPFLAGS="$EXTRA_HIPFLAGS" >/dev/null
mkdir -p "$D/lib"; mv "$D/pkg/lib/libgol.so" "$D/lib/"; rm -rf "$D/pkg/build"
echo "$D/lib/libgol.so"
