// direct.h -- the direct peer-memory transport (direct.cpp), internal.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <string>
#include <vector>

#include "bine_internal.h"

namespace bine {

// The flat reduce-scatter's tree fed by an exchange's receives, evaluated in
// the exchange's own launches (k_dm_move_tree): every receive is a leaf
// (`leaf_of_recv[i]` = its tree position), all of `leaf_bytes`; the tree of
// round r covers bytes [r * slot, ...) of every leaf, of `own_leaf` and of `out`.
struct TreeSpec {
  int nl = 0, pos = 0;
  unsigned swap = 0;
  std::vector<int> leaf_of_recv;
  const char *own_leaf = nullptr;
  char *out = nullptr;
  size_t leaf_bytes = 0;
  int dtype = 0, op = 0;
};

struct DirectState {
  int P = 1, rank = 0, device = 0;
  size_t slot = (size_t)64 << 20;  // sub-message size (BINE_DIRECT_SLOT_BYTES; profiles/r4_dm_stamps_p2_sweep2.txt)
  int wgs = 128;                   // workgroups per message (BINE_DIRECT_WGS; bine_comm_set_direct_wgs)
  int fused_wgs = 0;               // workgroups of a large call's single k_dm_fused launch (BINE_DIRECT_FUSED_WGS;
                                   // 0: tree_wgs -- every workgroup of that launch does tree work; cut to the
                                   // residency cap, then to a multiple of the CUs)
  int env_wgs = 128;               // the value init() settled on (the setter's 0)
  int pull_wgs = 0;                // workgroups per copied pull (BINE_DIRECT_PULL_WGS; 0: wgs)
  bool autoscale = true;           // a k_dm_move launch below the GPU's resident capacity scales its
                                   // messages' workgroups up (BINE_DIRECT_AUTOSCALE=0: off)
  // diagnostics (BINE_DIRECT_STAMPS=<records>): per-workgroup stamps of every
  // launch (DmArgs::stamps), read back with bine_comm_direct_stamps
  uint64_t *stamps = nullptr;
  uint32_t serial = 0;
  int merge = 3;                   // launch structure (BINE_DIRECT_MERGE): 2 = pushes + pulls of a round in one
                                   // launch, 1 = round k-1's pulls with round k's pushes, 0 = separate launches,
                                   // 3 = 2 for one-round exchanges, else 1
  uint64_t timeout_ticks = 0;      // wall_clock64 ticks of one wait (BINE_DIRECT_TIMEOUT_S, default 10 s)
  size_t data_off = 0, total = 0;
  hipMemGenericAllocationHandle_t own_h{};
  void *own = nullptr;
  int own_fd = -1;
  uint32_t *hpoison = nullptr;      // pinned host word: set with the device word on a timeout
  uint32_t *hpoison_dev = nullptr;  // its device-side address
  std::vector<void *> peer;  // peer[x] = x's inbox mapped here (peer[rank] = own)
  std::vector<hipMemGenericAllocationHandle_t> peer_h;

  ~DirectState();
  // phase 1, local: allocate the inbox, zero its flags, export its descriptor
  int init(int P, int rank, int device, std::string &err);
  // phase 2, collective over the P ranks of the node (same key on all):
  // exchange descriptors over Unix sockets, map every peer's inbox
  int connect_peers(uint64_t key, std::string &err);
  // tree: the receives r are the leaves of `tree`, evaluated in this
  // exchange's launches; dleaves + dtree: the receives of an EARLIER exchange
  // (issued there without them) are the leaves of `dtree`, pulled and
  // evaluated in this exchange's first launch, beside its own messages
  int exchange(const std::vector<XSend> &s, const std::vector<XRecv> &r, hipStream_t st,
               const TreeSpec *tree = nullptr, const std::vector<XRecv> *dleaves = nullptr,
               const TreeSpec *dtree = nullptr);
  // whether exchange() can take `tree` for these sends / receives (all of one
  // round's messages in one launch, 16-B vectors, an instantiated tree)
  bool tree_ok(const std::vector<XSend> &s, const std::vector<XRecv> &r, const TreeSpec &tree) const;
  // whether an exchange with these sends / receives can host the deferred
  // leaves of `dtree` (one slot each, all in its first launch)
  bool defer_ok(const std::vector<XSend> &s, const std::vector<XRecv> &r, const std::vector<XRecv> &dleaves,
                const TreeSpec &dtree) const;
  int tree_wgs = 256;  // tree workgroups per launch (BINE_DIRECT_TREE_WGS; bine_comm_set_direct_tree)
  int tree_wgs_env = 256;  // the value init() settled on
  // `share` ranks of this transport on this rank's GPU (more than one only
  // where several processes share a device; 1 on a node): the divisor of
  // every launch's residency cap (bine_internal.h dm_fit_residency), so the
  // co-located ranks' current launches are resident together.  Round 4's
  // share / 2 cut of the workgroup counts is subsumed by the cap.
  int share = 1;
  bool slice_flags = true;  // k_dm_fused's per-slice flags (BINE_DIRECT_SLICE_FLAGS=0: whole-message flags only)
  bool mcast = false;     // pushes of the same bytes to several peers as one group (BINE_DIRECT_MCAST=1;
                          // off: no gain measured, profiles/r3_push_groups.txt)
  bool poisoned() const { return hpoison && *(volatile uint32_t *)hpoison != 0; }
  int clock_khz = 0;  // wall_clock64 rate (the record's ticks -> seconds)
  // the timeout's cause: the first timed-out waiter's record (dm::kRecFirst,
  // mapped host words) and, with `flags`, per peer the ready / ack flags vs
  // this rank's sequence bases (device reads: only once the streams drained)
  std::string describe(bool flags) const;
  // stderr: describe(true)
  void dump() const;
  // the flag latency probe with `peer` (k_dm_ping; both ranks of the pair call
  // it together): *ticks = wall_clock64 ticks of round trips 2 .. iters, 0 when
  // the wait timed out (the transport is then poisoned)
  std::vector<uint64_t> ping_count;  // per peer: ping sequence numbers used so far (both ends count alike)
  uint64_t *ping_out = nullptr;      // device word the probe writes
  int ping(int peer, int iters, hipStream_t st, uint64_t *ticks);
};

}  // namespace bine
