# round-5 C3 stream-shape A/B with the held stream: MCEIK_PIPES 1 / 2 / 3 and the multi-step launch
# (MCEIK_PERSIST=1), interleaved rounds on one box; plus a sysfs probe of the node's GPUs.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${F_OUT:-r05pipes}
mkdir -p "$O"
( while sleep 45; do echo "[r05p] $(date +%T) running"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null || true' EXIT
python3 -c "import bench; print(bench.node_gpus())" > "$O/node_gpus.txt" 2>&1 || true
( ls /sys/class/kfd/kfd/topology/nodes 2>&1; for d in /sys/bus/pci/devices/*; do echo "$d $(cat $d/vendor) $(cat $d/class)"; done ) \
    > "$O/sysfs_probe.txt" 2>&1 || true
for r in 1 2; do
  for v in p1 p2 p3 ms; do
    case $v in p1) E="MCEIK_PIPES=1";; p2) E="MCEIK_PIPES=2";; p3) E="MCEIK_PIPES=3";; ms) E="MCEIK_PERSIST=1 MCEIK_PIPES=1";; esac
    P=${E##*MCEIK_PIPES=}
    env $E timeout -k 10 300 python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --f64-steps 0 --pipes $P \
        > "$O/${v}_r$r.log" 2>&1
    python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" \
        "$O/${v}_r$r.log" "$v" | tee -a "$O/summary.txt"
  done
done
echo done > "$O/DONE"
