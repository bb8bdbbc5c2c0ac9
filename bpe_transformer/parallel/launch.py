"""Single-node launcher: one process per GPU without ``torchrun``.

The reference declares ``submitit`` as its job launcher (``pyproject.toml:15``)
but never uses it.  Here ``launch(fn, nprocs)`` spawns ``nprocs`` fresh
interpreters (``spawn`` start method: no process inherits an initialised GPU
context, nothing is ``exec``'d after GPU init), exports the torchrun
environment (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 /
MASTER_PORT) in each child before ``fn`` runs, and re-raises the first
child failure in the parent.  ``fn`` then calls
:func:`bpe_transformer.parallel.init_distributed` as under torchrun.

CLI (runs a script's, or with ``-m`` a module's, ``__main__`` in every rank)::

    python -m bpe_transformer.parallel.launch --nproc 8 train.py --config ...
    python -m bpe_transformer.parallel.launch --nproc 8 -m bpe_transformer.train --preset gpt2-small
"""

from __future__ import annotations

import argparse
import os
import runpy
import socket
import sys
from typing import Any, Callable

import torch.multiprocessing as mp


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _child(local_rank: int, nprocs: int, port: int, fn: Callable, args: tuple, extra_env: dict) -> None:
    os.environ.update(extra_env)
    os.environ.update({"RANK": str(local_rank), "LOCAL_RANK": str(local_rank), "WORLD_SIZE": str(nprocs),
                       "LOCAL_WORLD_SIZE": str(nprocs), "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    fn(*args)


def launch(fn: Callable[..., Any], nprocs: int, *args: Any, port: int | None = None,
           env: dict[str, str] | None = None) -> None:
    """Run ``fn(*args)`` in ``nprocs`` ranks on this node and wait for all of them."""
    if nprocs < 1:
        raise ValueError("nprocs must be >= 1")
    extra = {"HSA_ENABLE_IPC_MODE_LEGACY": "0"}  # dmabuf IPC, required by RCCL on this platform
    extra.update(env or {})
    mp.start_processes(_child, args=(nprocs, port or free_port(), fn, args, extra), nprocs=nprocs, join=True,
                       start_method="spawn")


def _run_script(path: str, argv: list[str], module: bool = False) -> None:
    sys.argv = [path, *argv]
    if module:
        runpy.run_module(path, run_name="__main__", alter_sys=True)
    else:
        runpy.run_path(path, run_name="__main__")


def main(argv: list[str] | None = None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--nproc", type=int, default=1)
    ap.add_argument("--port", type=int, default=None)
    ap.add_argument("target", help="script path, or -m MODULE")
    # everything after the script / module name belongs to it
    split = next((i for i, t in enumerate(argv) if not t.startswith("--") and (i == 0 or argv[i - 1] not in
                  ("--nproc", "--port"))), len(argv))
    module = split < len(argv) and argv[split] == "-m"
    if module:
        if split + 1 >= len(argv):
            ap.error("-m needs a module name")
        own, target, rest = argv[:split], argv[split + 1], argv[split + 2:]
    else:
        own, target, rest = argv[:split], (argv[split] if split < len(argv) else None), argv[split + 1:]
    a = ap.parse_args(own + ([target] if target else []))
    launch(_run_script, a.nproc, a.target, rest, module, port=a.port)
    return 0


if __name__ == "__main__":
    sys.exit(main())
