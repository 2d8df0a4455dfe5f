"""Fail-safe multi-rank execution (the stage watchdog), the TCP rendezvous that
carries the RCCL unique id for El::Initialize, and the environment API the
drop-in header exposes (COMM_WORLD, the blocksize stack) — all on CPU.

The watchdog replaces the error fencing the reference gets from MPI / Aluminum
(include/El/core/imports/mpi/aluminum_comm.hpp:174-212): a stage that overruns
its deadline ends the process with a non-zero status naming the stage, instead
of leaving a multi-rank job hung."""
import os
import socket
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(ROOT, "tests", "_failsafe_worker.py")
WATCHDOG_EXIT = 75


def _port():
    """A free port below the ephemeral range (see tests/test_dist_cpu.py)."""
    import random
    for _ in range(200):
        p = random.randrange(20000, 32000)
        s = socket.socket()
        try:
            s.bind(("127.0.0.1", p))
            return p
        except OSError:
            continue
        finally:
            s.close()
    raise RuntimeError("no free port in 20000-32000")


def _run(*args, timeout=60):
    t0 = time.monotonic()
    p = subprocess.run([sys.executable, WORKER, *map(str, args)], capture_output=True, text=True, timeout=timeout)
    return p, time.monotonic() - t0


def test_watchdog_ends_an_overrunning_stage():
    p, dt = _run("deadline", "unit stage", 1.0, 30)
    assert p.returncode == WATCHDOG_EXIT, (p.returncode, p.stderr)
    assert "[elx] stage unit stage (deadline 1 s)" in p.stderr
    assert "FATAL in stage 'unit stage'" in p.stderr and "deadline of 1 s exceeded" in p.stderr
    assert "survived" not in p.stdout
    assert dt < 20


def test_watchdog_disarmed_stage_runs_to_the_end():
    p, _ = _run("disarm", 0.5, 1.5)
    assert p.returncode == 0, p.stderr
    assert "survived" in p.stdout and "[elx] stage disarmed" in p.stderr


def test_watchdog_gloo_world2_peer_never_joins():
    """Rank 0 blocks inside a 1x2 El::Gemm whose peer never enters it: the
    watchdog ends rank 0 at its 3 s deadline (stage named), and the straggler at
    its own — nobody hangs for gloo's 30-minute default."""
    port = _port()
    procs = [subprocess.Popen([sys.executable, WORKER, "gloo_hang", str(r), "2", str(port)],
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(2)]
    t0 = time.monotonic()
    outs = [p.communicate(timeout=90) for p in procs]
    dt = time.monotonic() - t0
    assert [p.returncode for p in procs] == [WATCHDOG_EXIT, WATCHDOG_EXIT], [o[1][-2000:] for o in outs]
    assert "FATAL in stage 'c3 timed'" in outs[0][1]
    assert "FATAL in stage 'straggler'" in outs[1][1]
    assert "gemm returned" not in outs[0][0]
    assert dt < 60


@pytest.mark.parametrize("world", [2, 3])
def test_rendezvous_bcast(world):
    port = _port()
    procs = [subprocess.Popen([sys.executable, WORKER, "rendezvous", str(r), str(world), str(port)],
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in reversed(range(world))]
    outs = [p.communicate(timeout=60) for p in procs]
    assert all(p.returncode == 0 for p in procs), [o[1] for o in outs]
    assert sorted(o[0].strip() for o in outs) == [f"rank {r} ok" for r in range(world)]


def test_rendezvous_ignores_stray_connections():
    """Stray connections to rank 0 (silent, garbage, a wrong world size, a
    duplicate rank) never use up a peer's slot: both real peers still get the
    id, and the strays get nothing."""
    import socket as so
    port = _port()
    root = subprocess.Popen([sys.executable, WORKER, "rendezvous", "0", "3", str(port)],
                            stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    strays = []
    deadline = time.monotonic() + 30
    while not strays:
        try:
            strays.append(so.create_connection(("127.0.0.1", port), timeout=2))
        except OSError:
            assert time.monotonic() < deadline
            time.sleep(0.05)
    import struct
    for payload in (b"GET / HTTP/1.0\r\n\r\n", b"ELXRDV02" + struct.pack("<iiQ", 1, 7, 0),
                    b"ELXRDV02" + struct.pack("<iiQ", 0, 3, 0), b"ELXRDV02" + struct.pack("<iiQ", 5, 3, 0),
                    b"ELXRDV01" + struct.pack("<ii", 1, 3)):
        c = so.create_connection(("127.0.0.1", port), timeout=2)
        c.sendall(payload)
        strays.append(c)
    peers = [subprocess.Popen([sys.executable, WORKER, "rendezvous", str(r), "3", str(port)],
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in (1, 2)]
    outs = [p.communicate(timeout=60) for p in [root] + peers]
    assert all(p.returncode == 0 for p in [root] + peers), [o[1] for o in outs]
    for c in strays:
        c.settimeout(2)
        try:
            assert c.recv(16) == b""  # closed without the payload
        except (so.timeout, ConnectionResetError):
            pass
        c.close()


def _fnv1a64(s: str) -> int:
    h = 14695981039346656037
    for b in s.encode():
        h = ((h ^ b) * 1099511628211) % (1 << 64)
    return h


def test_rendezvous_secret_and_loopback_bind():
    """ELX_RENDEZVOUS_SECRET: a well-formed hello for a real rank that carries
    another job's token (here: none) is refused and never takes that rank's
    slot; the peers holding the secret are served.  With MASTER_ADDR 127.0.0.1,
    rank 0 listens on the loopback address only, not on every interface."""
    import socket as so
    import struct
    import psutil
    port = _port()
    env = dict(os.environ, ELX_RENDEZVOUS_SECRET="job-4711")
    root = subprocess.Popen([sys.executable, WORKER, "rendezvous", "0", "3", str(port)], env=env,
                            stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    deadline = time.monotonic() + 30
    listen = []
    while not listen:
        assert time.monotonic() < deadline
        try:
            listen = [c for c in psutil.Process(root.pid).net_connections(kind="tcp")
                      if c.status == psutil.CONN_LISTEN and c.laddr.port == port]
        except psutil.NoSuchProcess:
            break
        time.sleep(0.05)
    assert [c.laddr.ip for c in listen] == ["127.0.0.1"], listen
    wrong = []
    for tok in (0, _fnv1a64("job-4712")):
        c = so.create_connection(("127.0.0.1", port), timeout=2)
        c.sendall(b"ELXRDV02" + struct.pack("<iiQ", 1, 3, tok))
        wrong.append(c)
    peers = [subprocess.Popen([sys.executable, WORKER, "rendezvous", str(r), "3", str(port)], env=env,
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in (1, 2)]
    outs = [p.communicate(timeout=60) for p in [root] + peers]
    assert all(p.returncode == 0 for p in [root] + peers), [o[1] for o in outs]
    for c in wrong:
        c.settimeout(2)
        try:
            assert c.recv(16) == b""
        except (so.timeout, ConnectionResetError):
            pass
        c.close()


def test_rendezvous_times_out_without_rank0():
    from elemental_amd import el
    from elemental_amd import _lib as L
    with pytest.raises(L.ElxError, match="could not reach rank 0"):
        el.rendezvous_bcast(None, 16, 1, 2, "127.0.0.1", _port(), 0.5)


def test_blocksize_stack_and_comm_world():
    """PushBlocksizeStack / PopBlocksizeStack / EmptyBlocksizeStack
    (environment/decl.hpp:88-94) and COMM_WORLD (size 1 without a launcher).
    The global stack is restored in `finally`, so a failing assertion here
    cannot leave later tests with an empty stack."""
    from elemental_amd import el
    from elemental_amd import _lib as L
    el.Initialize()
    try:
        assert el.Blocksize() == 128
        el.PushBlocksizeStack(64)
        assert el.Blocksize() == 64
        el.SetBlocksize(32)
        assert el.Blocksize() == 32
        el.PopBlocksizeStack()
        assert el.Blocksize() == 128
        el.EmptyBlocksizeStack()
        with pytest.raises(L.LogicError, match="empty stack"):
            el.Blocksize()
        with pytest.raises(L.LogicError, match="empty"):
            el.PopBlocksizeStack()
        el.PushBlocksizeStack(128)
        w = el.Comm.world()
        assert w.size == 1 and w.rank == 0
        g = el.Grid(w)
        assert (g.height, g.width) == (1, 1)
    finally:
        el.Finalize()
        el.EmptyBlocksizeStack()
        el.PushBlocksizeStack(128)  # Finalize empties the stack; later tests expect the default
    assert el.Blocksize() == 128
