"""Run bench.py with Python module flags overridden, for same-box end-to-end A/B runs without environment knobs.

    python benchmarks/bench_ab.py --set bpe_transformer.models.fused_block._FUSE_QKV_ROPE=0 -- --steps 20

Each ``--set module.attr=value`` imports the module and sets the attribute (ints / floats / True / False parsed,
anything else kept as a string) before bench.py runs in this process; each ``--op name=int`` calls the HIP
library's run-time switch ``torch.ops.bpe_hip.<name>(int)`` (e.g. ``--op fa_dq_config=1``); everything after
``--`` goes to bench.py.
"""
import importlib
import os
import runpy
import sys


def _parse(v: str):
    if v in ("True", "False"):
        return v == "True"
    for t in (int, float):
        try:
            return t(v)
        except ValueError:
            pass
    return v


def main():
    argv = sys.argv[1:]
    rest = []
    if "--" in argv:
        i = argv.index("--")
        argv, rest = argv[:i], argv[i + 1:]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    it = iter(argv)
    for a in it:
        if a == "--op":
            name, value = next(it).split("=", 1)
            import torch

            from bpe_transformer import ops

            ops.load()
            prev = getattr(torch.ops.bpe_hip, name)(int(value))
            print(f"[bench_ab] {name}({value}) (was {prev})", file=sys.stderr)
            continue
        if a != "--set":
            sys.exit(f"unknown argument {a!r} (use --set module.attr=value / --op name=int ... -- bench args)")
        spec = next(it)
        target, value = spec.split("=", 1)
        mod, attr = target.rsplit(".", 1)
        m = importlib.import_module(mod)
        if not hasattr(m, attr):
            sys.exit(f"{mod} has no attribute {attr}")
        setattr(m, attr, _parse(value))
        print(f"[bench_ab] {target} = {getattr(m, attr)!r}", file=sys.stderr)
    sys.argv = [os.path.join(root, "bench.py"), *rest]
    runpy.run_path(sys.argv[0], run_name="__main__")


if __name__ == "__main__":
    main()
