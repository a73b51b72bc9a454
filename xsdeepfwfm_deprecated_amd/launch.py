"""One process per GPU for a script's ``--gpus N`` (batch shards, one rank per device).

``spawn_ranks`` is called by a script's ``main()`` BEFORE anything touches the GPU: when the process was not
started by ``torch.distributed.run`` (``WORLD_SIZE`` unset) and N > 1 ranks are asked for, it starts the same
script N times as child processes with ``RANK`` / ``LOCAL_RANK`` / ``WORLD_SIZE`` / ``LOCAL_WORLD_SIZE`` /
``MASTER_ADDR=127.0.0.1`` / ``MASTER_PORT`` set (the environment ``torchrun --standalone`` gives its workers),
waits for all of them and returns the exit code for the parent to exit with; the parent itself never makes a
HIP call.  The children inherit stdout / stderr, so rank 0's JSON line is the parent's output.  If any rank
fails, the others are terminated (they would otherwise wait in a collective forever) and the parent's exit
code is non-zero.  Returns None in a rank (or when one process is enough): the caller then runs the work.
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import time


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n: int, argv=None, poll_s: float = 0.2, env_extra=None):
    """Run ``python <argv>`` as n ranks when this process is not already a rank; see the module docstring."""
    if n <= 1 or "WORLD_SIZE" in os.environ:
        return None
    argv = list(sys.argv if argv is None else argv)
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ)
        env.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(n), "LOCAL_WORLD_SIZE": str(n),
                    "GROUP_RANK": "0", "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this stack (RCCL)
        if env_extra:
            env.update(env_extra)
        procs.append(subprocess.Popen([sys.executable] + argv, env=env))
    rc = 0
    try:
        live = list(procs)
        while live:
            for p in list(live):
                code = p.poll()
                if code is None:
                    continue
                live.remove(p)
                if code != 0 and rc == 0:
                    rc = code if code > 0 else 128 - code  # a signal -> 128 + signal number
                    print(f"launch: rank {procs.index(p)} exited with {code}; stopping the other ranks",
                          file=sys.stderr, flush=True)
                    for q in live:
                        q.send_signal(signal.SIGTERM)
            if live:
                time.sleep(poll_s)
    finally:
        deadline = time.time() + 30
        for p in procs:
            if p.poll() is None:
                try:
                    p.wait(timeout=max(0.1, deadline - time.time()))
                except subprocess.TimeoutExpired:
                    p.kill()
                    p.wait()
    return rc
