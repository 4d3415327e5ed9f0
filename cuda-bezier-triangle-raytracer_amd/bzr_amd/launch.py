"""One process per GPU without an external launcher (bench.py --gpus N).

`python bench.py --gpus N` run bare (no WORLD_SIZE in the environment) starts N copies of itself as child
processes, rank r on LOCAL_RANK r, with a rendezvous on 127.0.0.1, waits for all of them and exits with the
first failing rank's status.  The parent imports nothing that touches the GPU (not even torch), so the
children own the devices; it never exec()s.  Under an external launcher (torch.distributed.run sets
WORLD_SIZE) nothing is spawned, and a WORLD_SIZE that disagrees with --gpus is an error: a bench line must
describe the ranks that actually ran.

Rays are independent (reference/test.cpp:376-401), so the ranks share nothing but the rendezvous and the
final gather of each frame.
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import threading
import time

LAUNCHED_BY = "BZR_LAUNCHED_BY"  # set in the children's environment: "bench.py" (self-launched)


def free_port() -> int:
    """A TCP port on 127.0.0.1 nobody listens on right now (the rendezvous port of the children)."""
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def check_world(gpus: int, env=None) -> str:
    """How this process's ranks come about: 'single' (gpus == 1, no launcher), 'spawn' (gpus > 1, no launcher:
    the caller must spawn()), 'launched' (WORLD_SIZE set and equal to gpus).  Raises SystemExit(2) when
    WORLD_SIZE is set and differs from gpus, or gpus < 1."""
    env = os.environ if env is None else env
    if gpus < 1:
        _die(f"bench.py: --gpus {gpus}: need at least one GPU")
    ws = env.get("WORLD_SIZE")
    if ws is None or ws == "":
        return "spawn" if gpus > 1 else "single"
    if not ws.isdigit() or int(ws) != gpus:
        _die(f"bench.py: --gpus {gpus} but WORLD_SIZE={ws}: the launcher started a different number of ranks "
             f"than the line would report; pass --gpus {ws} (or run without a launcher)")
    return "launched"


def _die(msg: str):
    print(msg, file=sys.stderr, flush=True)
    raise SystemExit(2)


def spawn(argv: list[str], n: int, env=None, master_addr: str = "127.0.0.1", poll_s: float = 0.05) -> int:
    """Run `argv` (a full command line, e.g. [sys.executable, 'bench.py', ...]) as n ranks: RANK = LOCAL_RANK =
    r, WORLD_SIZE = n, MASTER_ADDR / MASTER_PORT for the rendezvous.  Returns 0 when every rank exits 0,
    else the first failing rank's exit status (a signal -s maps to 128 + s); once a rank fails the others
    get SIGTERM (they would otherwise wait in a collective for it), then SIGKILL after 15 s."""
    base = dict(os.environ if env is None else env)
    base.update(MASTER_ADDR=master_addr, MASTER_PORT=str(free_port()), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n))
    base[LAUNCHED_BY] = "bench.py"
    procs = []
    try:
        for r in range(n):
            e = dict(base, RANK=str(r), LOCAL_RANK=str(r))
            procs.append(subprocess.Popen(argv, env=e))
    except OSError:
        for p in procs:
            p.kill()
        raise
    status, failed_at = 0, None
    live = set(range(n))

    def on_term(signum, frame):  # a SIGTERM to the parent unwinds through the finally below
        raise SystemExit(128 + signum)

    old_term = signal.signal(signal.SIGTERM, on_term) if threading.current_thread() is threading.main_thread() else None
    try:
        while live:
            for r in sorted(live):
                rc = procs[r].poll()
                if rc is None:
                    continue
                live.discard(r)
                if rc != 0 and status == 0:
                    status = rc if rc > 0 else 128 - rc
                    failed_at = time.monotonic()
                    print(f"bench.py: rank {r} exited with status {rc}; stopping the other ranks", file=sys.stderr, flush=True)
                    for q in live:
                        procs[q].send_signal(signal.SIGTERM)
            if failed_at is not None and live and time.monotonic() - failed_at > 15.0:
                for q in live:
                    procs[q].kill()
            time.sleep(poll_s)
    finally:  # the parent interrupted (KeyboardInterrupt, SIGTERM): no rank outlives it
        _stop([procs[q] for q in live])
        if old_term is not None:
            signal.signal(signal.SIGTERM, old_term)
    return status


def _stop(procs, grace_s: float = 15.0):
    """SIGTERM the running children, SIGKILL those still running after `grace_s`, and reap them."""
    running = [p for p in procs if p.poll() is None]
    for p in running:
        p.send_signal(signal.SIGTERM)
    deadline = time.monotonic() + grace_s
    for p in running:
        try:
            p.wait(timeout=max(0.0, deadline - time.monotonic()))
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()
