#!/bin/bash
# Run the reference's pico_core against the MI355X libbine.so drop-in.
#   usage: integration/run_pico_core.sh NP COLLECTIVE COUNT ITER ALGO DTYPE [SEGSIZE]
#   e.g.   integration/run_pico_core.sh 1 ALLREDUCE 67108864 20 bine_bdw_remap_over float
# pico_core checks every result against the MPI library's own PMPI_* collective
# (pico_core_utils.c:553-610) and aborts on mismatch.
set -e
HERE="$(cd "$(dirname "$0")" && pwd)"
NP=$1; COLL=$2; COUNT=$3; ITER=$4; ALGO=$5; DT=$6; SEG=${7:-0}
OUT="${PICO_OUT:-$HERE/../gpurun_out/pico_core}"
mkdir -p "$OUT/data"
export COLLECTIVE_TYPE=$COLL OUTPUT_DIR="$OUT" DATA_DIR="$OUT/data" OUTPUT_LEVEL=all LOCATION=local
if [ "$SEG" != "0" ]; then export SEGMENTED=yes SEGSIZE=$SEG; else export SEGMENTED=no; fi
export PATH=/opt/conda/bin:$PATH
if [ "$NP" -gt 1 ] && [ -n "$BINE_FAKE_HOSTS" ]; then
  # several ranks on ONE GPU: give each a different RCCL host id (socket transport)
  args=()
  for ((r = 0; r < NP; r++)); do
    [ $r -gt 0 ] && args+=(":")
    args+=(-n 1 -env NCCL_HOSTID "fake-host-$r" -env NCCL_SOCKET_IFNAME lo "$HERE/_build/pico_core" "$COUNT" "$ITER" "$ALGO" "$DT")
  done
  exec mpiexec "${args[@]}"
fi
exec mpiexec -n "$NP" "$HERE/_build/pico_core" "$COUNT" "$ITER" "$ALGO" "$DT"
