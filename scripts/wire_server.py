"""Run a wire front end (wire.py's ClusterTokenServer, or --native: sentinel_wire_server) on config-2
rules for a load test.

BASELINE config 2: 10k flowIds (1..F), GLOBAL, count ~ U{10..1000}, sampleCount 2 / 1000 ms.  Writes
the listening port to --port-file, serves for --seconds, then prints the server's batch count.
usage: python scripts/wire_server.py --port-file P [--seconds S] [--flows F] [--max-wait-ms W]"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import sentinel_amd as sa                        # noqa: E402
from sentinel_amd import wire as W               # noqa: E402
from sentinel_amd.token_service import ServerNamespace   # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--port-file", required=True)
    ap.add_argument("--seconds", type=float, default=120.0, help="serve at most this long")
    ap.add_argument("--stop-file", default=None, help="stop as soon as this file exists")
    ap.add_argument("--flows", type=int, default=10000)
    ap.add_argument("--max-wait-ms", type=float, default=0.2)
    ap.add_argument("--max-batch", type=int, default=65536)
    ap.add_argument("--native", action="store_true", help="sentinel_wire_server (C++) instead of wire.py")
    ap.add_argument("--io-threads", type=int, default=4)
    ap.add_argument("--max-wait-us", type=int, default=20)
    a = ap.parse_args()
    rng = np.random.default_rng(2)
    F = a.flows
    svc = sa.GpuTokenService(0)
    svc.set_namespaces([ServerNamespace(connected_count=1)])
    svc.load_rules_array(np.arange(1, F + 1, dtype=np.int64), rng.integers(10, 1001, F).astype(np.float64),
                         np.ones(F, np.int32), np.full(F, 2, np.int32), np.full(F, 1000, np.int32),
                         np.zeros(F, np.int32), np.zeros(F, np.int32))
    if a.native:
        srv = W.NativeTokenServer(svc, io_threads=a.io_threads, max_batch=min(a.max_batch, 4096),
                                  max_wait_us=a.max_wait_us)
    else:
        srv = W.ClusterTokenServer(svc, max_batch=a.max_batch, max_wait_ms=a.max_wait_ms)
    port = srv.port if a.native else srv.start()
    with open(a.port_file + ".tmp", "w") as f:
        f.write(str(port))
    os.replace(a.port_file + ".tmp", a.port_file)
    t_end = time.time() + a.seconds
    while time.time() < t_end and not (a.stop_file and os.path.exists(a.stop_file)):
        time.sleep(0.1)
    if a.native:
        st = srv.stats()
        srv.stop()
        print(json.dumps({"server": "native", "io_threads": a.io_threads, "max_wait_us": a.max_wait_us, **st}), flush=True)
    else:
        srv.stop()
        print(json.dumps({"server": "wire.py", "batches": srv.batches, "max_wait_ms": a.max_wait_ms}), flush=True)


if __name__ == "__main__":
    main()
