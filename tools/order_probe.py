"""Order probe: ms/step of a sequence of bench configs run in ONE process (bench.run_config,
5 timed steps or $STEPS, 2 warmup, lanes per config or $PIPE), e.g. `python tools/order_probe.py C2 C2 C2` or `C1 C2`."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    pkg = bench.entry.load_package()
    env = bench.Env(1)
    for cfg in sys.argv[1:]:
        steps = int(os.environ.get("STEPS", "5"))
        pipe = os.environ.get("PIPE")
        r = bench.run_config(pkg, env, cfg, steps, 2, pipeline=int(pipe) if pipe else None)
        print(cfg, r["ms_per_step"], flush=True)


if __name__ == "__main__":
    main()
