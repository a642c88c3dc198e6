"""bench.py's sharded-leg watchdog must end a hung run with a non-zero status
(VERDICT r02 weak #6): a hung collective on the driver's multi-GPU run must not
read as rc = 0. CPU only: the watchdog is exercised in a child process."""
import os
import subprocess
import sys
import threading

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import sys, threading, time
sys.path.insert(0, sys.argv[1])
import bench
done = threading.Event()
threading.Thread(target=bench.watchdog, args=(done, 0.2, 0, lambda: print("HEADLINE", flush=True)),
                 daemon=True).start()
time.sleep(30)  # a 'hung collective'
"""


def test_watchdog_exits_nonzero_on_hang():
    r = subprocess.run([sys.executable, "-c", CHILD, ROOT], capture_output=True, text=True, timeout=60)
    import bench
    assert r.returncode == bench.WATCHDOG_EXIT != 0
    assert "HEADLINE" in r.stdout  # rank 0 still prints the line it has
    assert "exceeded" in r.stderr


def test_watchdog_quiet_when_done():
    sys.path.insert(0, ROOT)
    import bench
    done = threading.Event()
    done.set()
    calls = []
    bench.watchdog(done, 0.01, 0, exit_fn=calls.append)
    assert calls == []
