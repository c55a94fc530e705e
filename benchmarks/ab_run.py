"""A/B driver: flip native runtime setters, then run bench.py's main in this process.

    python benchmarks/ab_run.py --set head_score_pool_set=0 -- --steps 50 --warmup 10

Each ``--set NAME=INT`` calls ``torch.ops.fedrec.NAME(INT)`` before the bench starts (the
kernels' A/B switches are runtime setters, not environment knobs).  Everything after ``--``
goes to bench.py."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> int:
    argv = sys.argv[1:]
    rest = []
    if "--" in argv:
        i = argv.index("--")
        argv, rest = argv[:i], argv[i + 1:]
    sets = []
    while argv:
        a = argv.pop(0)
        if a == "--set":
            name, val = argv.pop(0).split("=")
            sets.append((name, int(val)))
        else:
            rest.insert(0, a)
    from fedrec_with_pytorchdistributed_amd.ops import native

    lib = native.lib()
    for name, val in sets:
        getattr(lib, name)(val)
        print(f"[ab_run] {name}({val})", file=sys.stderr, flush=True)
    import bench

    sys.argv = ["bench.py", *rest]
    return bench.main()


if __name__ == "__main__":
    sys.exit(main())
