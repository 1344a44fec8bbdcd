"""Generate tests/golden/bench_<W>.json (square boards) or
bench_<W>x<H>.json: the global state hash of one of bench.py's boards after
every generation, from the CPU oracle.

Tables committed (every board bench.py times carries a parity check):
  bench_262144.json        the headline 262144^2 board (and its N-rank shards,
                           and the whole-board self-ring window), epochs 0..140
  bench_65536.json         the 65536^2 roofline board (configs[2]): its short
                           window, the 1024-generation window and the
                           single-generation-pass window, epochs 0..1100
  bench_262144x32768.json  one rank's shard of the N = 8 decomposition as a
                           1-rank self-ring (a 262144 x 32768 torus; the
                           seed is counter-based on the global row, so its
                           rows are the big board's first 32768), epochs 0..140

bench.py's headline workload is the W x W torus, B3/S23, seeded with the
splitmix64 board of seed 0x5EED (BASELINE.json configs[3]).  The hash is
sharding-invariant, so the same table checks the whole
board on one GPU and the sum of N shards' partial hashes.  bench.py looks up
the epoch its board reached (W + K generations, and 2 (W + K) after the
hashed window) and reports parity.match.

PARITY UNPINNED: like golden.json these vectors come from the oracle
restatement (oracle/gol_oracle.c), not from the reference, which has no tests
and cannot run here.  The seed and the hash are
cross-checked against the independent numpy restatement (oracle.np_seed,
oracle.np_hash) on row blocks of the board at epoch 0 and at the last epoch
(the hash is a sum over rows, so block hashes add up to the board's).

    python tests/golden/make_bench_golden.py [--board 262144] [--height H] [--gens 140] [--threads 8]

262144^2 needs 16 GiB of host memory (two 8 GiB planes) and ~25 min on 8
cores for 140 generations.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402

SEED = 0x5EED


def block_check(board: np.ndarray, W: int, rows: list[int], n: int = 64) -> None:
    """C hash == numpy hash on n-row blocks starting at `rows`."""
    for r0 in rows:
        blk = board[r0:r0 + n]
        c = O.hash_packed(blk, W, row0=r0)
        p = O.np_hash(blk, W, row0=r0)
        if c != p:
            raise SystemExit(f"C and numpy hashes disagree on rows {r0}..{r0 + n}: {c:#x} vs {p:#x}")


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--board", type=int, default=262144)
    ap.add_argument("--height", type=int, default=0, help="rows (0: square board)")
    ap.add_argument("--gens", type=int, default=140)
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 1)
    a = ap.parse_args()
    W = a.board
    H = a.height or a.board
    name = f"bench_{W}.json" if H == W else f"bench_{W}x{H}.json"
    out_path = os.path.join(os.path.dirname(os.path.abspath(__file__)), name)
    ww = O.wwords(W)
    L = O.lib()

    t0 = time.time()
    cur = O.seed_packed(W, H, SEED)
    nseed = min(H, 256)
    if not (O.np_seed(W, nseed, SEED) == cur[:nseed]).all():
        raise SystemExit("C and numpy seeds disagree")
    probe = [0, H // 2 - 32, H - 64]
    block_check(cur, W, probe)
    nxt = np.empty_like(cur)
    hashes = [O.hash_packed(cur, W)]
    print(f"seeded {W}x{H} in {time.time() - t0:.1f} s, epoch 0 hash {hashes[0]:#018x}", flush=True)

    u32p = O._u32p
    for g in range(1, a.gens + 1):
        L.oracle_step_packed(cur.ctypes.data_as(u32p), nxt.ctypes.data_as(u32p), W, H, ww, O.TORUS,
                             O.LIFE[0], O.LIFE[1], W, H, a.threads)
        cur, nxt = nxt, cur
        hashes.append(int(L.oracle_hash_packed(cur.ctypes.data_as(u32p), ww, 0, H, ww)))
        if g % 5 == 0 or g == a.gens:
            print(f"epoch {g}: {hashes[-1]:#018x}  ({time.time() - t0:.0f} s)", flush=True)
    block_check(cur, W, probe)

    doc = {
        "generator": "tests/golden/make_bench_golden.py (oracle/gol_oracle.c oracle_step_packed + "
                     "oracle_hash_packed; seed and block hashes cross-checked with numpy)",
        "parity": "unpinned (the reference ships no vectors; SURVEY.md section 0)",
        "board": [W, H], "topology": "torus", "rule": "B3/S23", "seed": SEED,
        "hash": "global state hash (DESIGN.md section 5), sum of shard partials mod 2^64",
        "hashes": [f"{h:#018x}" for h in hashes],
        "popcount_final": int(np.unpackbits(cur.view(np.uint8)).sum(dtype=np.int64)) if W <= 65536 else None,
    }
    with open(out_path, "w") as f:
        json.dump(doc, f, indent=1)
        f.write("\n")
    print(f"wrote {out_path}: epochs 0..{a.gens} in {time.time() - t0:.0f} s", flush=True)


if __name__ == "__main__":
    main()
