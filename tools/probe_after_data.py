"""Config 5 step rate in the same process right after bench.py's config-4 data leg (development
tool): isolates whether the data leg leaves state that slows the MLP leg.

    python tools/probe_after_data.py [steps]
"""
import os
import sys
import types

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import bench  # noqa: E402
import probe_mlp  # noqa: E402

if __name__ == "__main__":
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    probe_mlp.run(2000, True, True)
    args = types.SimpleNamespace(d=1000, n=1_000_000, seed=0, steps=K, warmup=2, profile_reps=3)
    r = bench.bench_data(args, 1, 0, 0)
    print(f"data leg: {r['value']:.2f} steps/s", flush=True)
    for _ in range(3):
        probe_mlp.run(2000, True, True)
