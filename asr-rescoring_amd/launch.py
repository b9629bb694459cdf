"""One process per GPU without an external launcher: ``bench.py --gpus N``.

``torch.distributed.run`` is the usual launcher (the driver's N > 1 runs use it).  When a
program is started directly with ``--gpus N`` (N > 1) and no ``WORLD_SIZE`` in the environment,
``spawn_ranks`` starts N fresh child processes of the same program with the rendezvous
variables torchrun would set (``RANK``, ``LOCAL_RANK``, ``WORLD_SIZE``, ``LOCAL_WORLD_SIZE``,
``MASTER_ADDR`` = 127.0.0.1, ``MASTER_PORT`` = a free port), relays rank 0's JSON lines (those
starting with ``{``) to its own stdout — every other line of every rank, including what native
libraries print to fd 1 (gloo, RCCL), goes to stderr, so exactly the result line comes back — and
returns the first failing rank's exit status.  If one rank fails, the others are terminated
(by their own process handles) instead of being left waiting at a collective.

The parent makes no GPU call: this module imports neither torch nor the library, and callers
must invoke it before anything initialises HIP (no exec: the children are new processes).
The reference scores in one process (``MLM_PLL/main.py:164-203``); the utterance-sharded
N-rank form is SURVEY §8(e).
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys
import threading
import time
from typing import List, Optional, Sequence

RANK_VARS = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")


def need_spawn(n: int, env=None) -> bool:
    """True when ``n`` ranks were asked for and no launcher has set up this process's rank."""
    env = os.environ if env is None else env
    return n > 1 and "WORLD_SIZE" not in env


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_env(rank: int, world: int, port: int, base=None) -> dict:
    env = dict(os.environ if base is None else base)
    env.update({"RANK": str(rank), "LOCAL_RANK": str(rank), "WORLD_SIZE": str(world),
                "LOCAL_WORLD_SIZE": str(world), "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    return env


def _pump(src, dst, rest):
    for line in iter(src.readline, b""):
        text = line.decode(errors="replace")
        d = dst if (dst is not None and text.lstrip().startswith("{")) else rest
        d.write(text)
        d.flush()
    src.close()


def spawn_ranks(n: int, argv: Sequence[str], script: Optional[str] = None, stdout=None,
                port: Optional[int] = None, poll_s: float = 0.2, grace_s: float = 20.0) -> int:
    """Run ``python script *argv`` (or ``python *argv`` with ``script=None``) as ``n`` ranks on
    127.0.0.1; returns 0 when every rank exits 0, else the first failing rank's status."""
    out = sys.stdout if stdout is None else stdout
    port = free_port() if port is None else port
    cmd = [sys.executable] + ([script] if script else []) + list(argv)
    procs: List[subprocess.Popen] = []
    pumps = []
    try:
        for r in range(n):
            p = subprocess.Popen(cmd, env=rank_env(r, n, port), stdout=subprocess.PIPE)
            procs.append(p)
            t = threading.Thread(target=_pump, args=(p.stdout, out if r == 0 else None, sys.stderr), daemon=True)
            t.start()
            pumps.append(t)
        status = 0
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                status = bad[0]
                break
            if all(c == 0 for c in codes):
                break
            time.sleep(poll_s)
    finally:
        for p in procs:                      # a failed rank: end the others (exact handles)
            if p.poll() is None:
                p.terminate()
        deadline = time.time() + grace_s
        for p in procs:
            try:
                p.wait(timeout=max(0.1, deadline - time.time()))
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
        for t in pumps:
            t.join(timeout=5)
    return status
