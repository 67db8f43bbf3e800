#!/bin/bash
# Run integration/op_check (the drop-in's MPI-typed entry points vs MPICH's
# own collectives) at NP ranks.  With BINE_FAKE_HOSTS set, several ranks share
# ONE GPU, each with its own RCCL host id (socket transport), as run_pico_core.sh.
#   usage: integration/run_op_check.sh NP [PROGRAM]   (PROGRAM: op_check (default) or buffer_churn)
set -e
HERE="$(cd "$(dirname "$0")" && pwd)"
NP=$1
PROG=${2:-op_check}
export PATH=/opt/conda/bin:$PATH
if [ "$NP" -gt 1 ] && [ -n "$BINE_FAKE_HOSTS" ]; then
  args=()
  for ((r = 0; r < NP; r++)); do
    [ $r -gt 0 ] && args+=(":")
    args+=(-n 1 -env NCCL_HOSTID "fake-host-$r" -env NCCL_SOCKET_IFNAME lo "$HERE/_build/$PROG")
  done
  exec mpiexec "${args[@]}"
fi
exec mpiexec -n "$NP" "$HERE/_build/$PROG"
