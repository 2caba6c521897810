#!/bin/bash
# Drop-in path measurements on the GPU box: the native batcher under T = 2 x cores synchronous
# callers and under async in-flight callers (tools/dropin_bench), then the wire front end over
# loopback TCP (scripts/wire_server.py + tools/wire_client).  Results: gpurun_out/dropin/*.json
set -e
OUT=gpurun_out/dropin
mkdir -p $OUT
CORES=${DROPIN_CORES:-16}
if [ -z "$ONLY_NATIVE" ]; then
timeout -k 10 60 tools/dropin_bench --mode sync --threads $((2 * CORES)) --seconds 5 > $OUT/batcher_sync.json
timeout -k 10 60 tools/dropin_bench --mode async --threads 4 --inflight 1024 --seconds 5 > $OUT/batcher_async.json
rm -f $OUT/port $OUT/stop
python -u scripts/wire_server.py --port-file $OUT/port --stop-file $OUT/stop --seconds 150 > $OUT/wire_server.log 2>&1 &
SRV=$!
for i in $(seq 1 120); do [ -f $OUT/port ] && break; sleep 1; done
PORT=$(cat $OUT/port)
rc=0
timeout -k 10 60 tools/wire_client --port $PORT --conns 16 --inflight 256 --seconds 5 > $OUT/wire_py.json || rc=$?
touch $OUT/stop
wait $SRV || true
[ $rc -eq 0 ] || exit $rc
fi
rc=0
# the native server: the same load, then more connections / deeper pipelines
rm -f $OUT/port $OUT/stop
python -u scripts/wire_server.py --native --io-threads ${IO_THREADS:-4} --port-file $OUT/port --stop-file $OUT/stop --seconds 150 > $OUT/wire_native_server.log 2>&1 &
SRV=$!
for i in $(seq 1 120); do [ -f $OUT/port ] && break; kill -0 $SRV 2>/dev/null || break; sleep 1; done
[ -f $OUT/port ] || { tail -5 $OUT/wire_native_server.log; exit 1; }
PORT=$(cat $OUT/port)
timeout -k 10 60 tools/wire_client --port $PORT --conns 16 --inflight 256 --seconds 5 > $OUT/wire_native.json || rc=$?
[ $rc -eq 0 ] && { timeout -k 10 60 tools/wire_client --port $PORT --conns 64 --inflight 1024 --seconds 5 > $OUT/wire_native_deep.json || rc=$?; }
[ $rc -eq 0 ] && { timeout -k 10 60 tools/wire_client --port $PORT --conns 32 --inflight 1 --seconds 5 > $OUT/wire_native_sync.json || rc=$?; }
touch $OUT/stop
wait $SRV || true
exit $rc
