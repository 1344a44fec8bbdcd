#!/usr/bin/env python3
"""In-kernel clock probe: its clock beside the kernel time with the probe on
and off (GOL_CLOCK_PROBE=0 in a second process), same box, reseeded board.

    python scripts/clock_probe_ab.py [WxH ...]   env: GPP=12,8  GENS=48
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "akka-game-of-life_amd"))

from gameoflife.engine import GolEngine  # noqa: E402


def main():
    shapes = [tuple(int(x) for x in a.split("x")) for a in sys.argv[1:]] or [(262144, 262144), (65536, 65536)]
    gpps = [int(g) for g in os.environ.get("GPP", "12,8").split(",")]
    gens = int(os.environ.get("GENS", "48"))
    tag = "probe-off" if os.environ.get("GOL_CLOCK_PROBE") == "0" else "probe-on"
    for W, H in shapes:
        with GolEngine(W, H) as e:
            for G in gpps:
                for rep in range(2):
                    e.set_tuning(gens_per_pass=G)
                    e.seed(0x5EED)
                    e.step(G)
                    e.sync()
                    e.profile(True)
                    e.profile_reset()
                    e.step(gens)
                    ms, n, g = e.profile_read()
                    clk = e.profile_clock()
                    e.profile(False)
                    print(f"{tag} {W}x{H} G={G} rep={rep} kernel_ms/gen={ms / g:.4f} probe_clock={clk:.3f} GHz",
                          flush=True)


if __name__ == "__main__":
    main()
