import os, sys, time
sys.path.insert(0, "/root/repo/akka-game-of-life_amd")
from gameoflife.engine import GolEngine
for (W, H, band) in [(4096, 4096, 0), (2048, 4096, 4), (2048, 4096, 0), (4096, 4096, 4)]:
    with GolEngine(W, H) as e:
        e.seed(0x5EED)
        e.set_tuning(band_rows=band, gens_per_pass=10)
        for hashed in (False, True):
            e.step(100, hashes=hashed); e.sync()
            best = 1e9
            for _ in range(3):
                t0 = time.perf_counter(); e.step(1000, hashes=hashed); e.sync(); best = min(best, time.perf_counter() - t0)
            print(f"{W}x{H} band={band or 'auto'} hash={int(hashed)} wall_ms={best*1e3:.3f} us/launch={best*1e6/100:.2f}", flush=True)
