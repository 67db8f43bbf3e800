"""Host-only model of the direct peer-memory transport's protocol
(pico_amd/csrc/direct.cpp) driven by the executor's real issue schedules
(bine_plan_schedule): every rank's comm and compute streams, the cross-stream
waits of the schedule, and per exchange the push / pull launches of each round
with their flag waits (push: ack >= seq - SLOTS; pull: ready >= seq) and
publications.  Messages of a started launch progress independently; a launch
completes when all its messages have.  Runs a few consecutive collectives and
reports a deadlock (no message or op can make progress) with the state.

Used by tests/test_direct_protocol.py (CPU).  Mirrors DirectState::exchange:
per peer, sequence numbers in the order the executor lists sends / receives;
messages cut into sub-messages of SLOT bytes, round k = k-th sub-message.
"""
from __future__ import annotations

import pico_amd

SLOTS = 4


def exchange_launches(rank, sends, recvs, seq_s, seq_r, slot, P, merge=3, deferred=(), mcast=True):
    """DirectState::exchange for one exchange: list of launches, each a list
    of messages {kind, peer, seq}.  `deferred`: an earlier exchange's leaf
    receives (one slot each) pulled at the start of the first launch"""
    maxb = max([x[1] for x in sends] + [b for _, b in recvs] + [0])
    rounds = (maxb + slot - 1) // slot
    out = []
    pre = []
    for p, _ in deferred:
        seq_r[p] += 1
        pre.append({"kind": "pull", "peer": p, "seq": seq_r[p]})
    ns, nr = [0] * P, [0] * P
    for x in sends:
        p = x[0]
        ns[p] += 1
        assert ns[p] <= SLOTS, "more messages to one peer than slots: refused by the library"
    for p, _ in recvs:
        nr[p] += 1
        assert nr[p] <= SLOTS
    def pushes(k):
        # sends of the same source and size in one launch form a group (the
        # library's multicast push: one set of workgroups waits for every
        # member's acknowledgement, then writes all of them)
        out = []
        for x in sends:
            p, b = x[0], x[1]
            if b > k * slot:
                seq_s[p] += 1
                m = {"kind": "push", "peer": p, "seq": seq_s[p]}
                if len(x) > 2 and mcast:
                    m["grp"] = (x[2], b, k)
                out.append(m)
        return out

    def pulls(k):
        out = []
        for p, b in recvs:
            if b > k * slot:
                seq_r[p] += 1
                out.append({"kind": "pull", "peer": p, "seq": seq_r[p]})
        return out

    # merge 2: launch k = round k's pushes + round k's pulls; merge 1: round
    # k-1's pulls + round k's pushes; merge 0: separate launches; merge 3
    # (the library's default): 2 for one round, else 1
    if merge == 2 or (merge == 3 and rounds == 1):
        for k in range(rounds):
            launch = (pre if k == 0 else []) + pushes(k) + pulls(k)
            if launch:
                out.append(launch)
        if rounds == 0 and pre:
            out.append(pre)
        return out
    for k in range(rounds + 1):
        launch = pulls(k - 1) if k > 0 else list(pre)
        if not merge and launch:
            out.append(launch)
            launch = []
        if k < rounds:
            launch = launch + pushes(k)
        if launch:
            out.append(launch)
    return out


def dm_tree_src(ops, i):
    """the tree op fed by exchange i: the first local op after it"""
    j = i + 1
    while j < len(ops) and ops[j]["xchg"]:
        j += 1
    return j


def dm_tree_plan(ops, esz, slot, kmax=32):
    """tests' restatement of the executor's plan_dm_trees (executor.cpp) on
    symbolic ranges (buffer, element offset, count): {tree op j: host
    exchange}, {exchange i: deferred}"""
    n = len(ops)

    def ranges(o, kind):
        return [(p["src_buf"] if kind == "SEND" else p["dst_buf"],
                 p["src_off"] if kind == "SEND" else p["dst_off"], p["count"]) for p in o["prims"]
                if p["type"] == kind]

    def ov(a, b):
        return a[0] == b[0] and a[1] < b[1] + b[2] and b[1] < a[1] + a[2]

    host, hosted, defer = {}, {}, set()
    for i in range(n):
        if not ops[i]["xchg"]:
            continue
        j = i + 1
        while j < n and ops[j]["xchg"]:
            j += 1
        if j >= n or ops[j]["wait"] != i or len(ops[j]["prims"]) != 1 or ops[j]["prims"][0]["type"] != "REDUCE_TREE":
            continue
        t = ops[j]["prims"][0]
        clean = all(not ((x["type"] not in ("REDUCE_TREE", "RECV") and x["src_buf"] == t["src_buf"])
                         or x["aux_buf"] == t["src_buf"] or (x["type"] != "RECV" and x["dst_buf"] == t["src_buf"]))
                    for o in ops for x in o["prims"])
        recvs = [p for p in ops[i]["prims"] if p["type"] == "RECV"]
        ok = clean and t["peer"] >= 2 and len(recvs) == t["peer"] - 1 and all(
            p["dst_buf"] == t["src_buf"] and p["count"] == t["count"] and p["dst_off"] >= t["src_off"]
            and (p["dst_off"] - t["src_off"]) % t["count"] == 0 for p in recvs)
        if not ok:
            continue
        out = (t["dst_buf"], t["dst_off"], t["count"])
        own = (t["aux_buf"], t["aux_off"], t["count"])
        i2 = i + 1
        while i2 < n and not ops[i2]["xchg"]:
            i2 += 1
        lb = t["count"] * esz
        # the tree reads / writes whole 16-B vectors from 16-B aligned own leaf and output
        if (t["aux_off"] * esz) % 16 or (t["dst_off"] * esz) % 16 or t["peer"] not in (2, 4, 8, 16):
            continue
        dfr = (i2 < n and ((i2 == i + 1 and i2 < j) or i2 == j + 1) and i2 not in hosted and ops[i2]["wait"] != j
               and lb <= slot and lb % 16 == 0)
        if dfr:
            s2, r2 = ranges(ops[i2], "SEND"), ranges(ops[i2], "RECV")
            dfr = not any(ov(x, out) for x in s2) and not any(ov(x, out) or ov(x, own) for x in r2)
            maxb = max([x[2] * esz for x in s2 + r2] + [0])
            dfr = dfr and len(recvs) + len(s2) + (len(r2) if maxb <= slot else 0) <= kmax
        if dfr:
            host[j] = i2
            hosted[i2] = j
            defer.add(i)
            continue
        if i not in hosted:
            s1 = ranges(ops[i], "SEND")
            if not any(ov(x, out) for x in s1) and len(s1) + len(recvs) <= kmax and lb % 16 == 0:
                host[j] = i
                hosted[i] = j
                continue
        if lb <= slot and lb % 16 == 0 and len(recvs) <= kmax:
            # a launch of its own at the tree's place (the tree op hosts itself)
            host[j] = j
            hosted[j] = j
            defer.add(i)
    return host, hosted, defer


def run(coll, algo, P, count=0, rcounts=None, esz=4, chunk_bytes=16 << 20, relay_min_bytes=0, trees=False,
        flat_ag=False, flat_rs=False, calls=3, slot=16 << 20, merge=3, dm_trees=False, stats=None,
        residency=None):
    """simulate `calls` consecutive collectives on all ranks; returns None if
    every one completes, else a description of the deadlock.  dm_trees: the
    flat reduce-scatter's trees fused into exchange launches as the executor
    does over the direct transport (deferred leaf pulls; `stats` counts them).

    residency (None: every workgroup of a started launch is resident, i.e. the
    protocol alone): {"gpu_of": [gpu of rank r], "slots": workgroup slots per
    GPU, "wgs": workgroups per message, "cap": True to apply the library's
    residency cut (dm_fit_residency: a launch's workgroups scaled to
    slots / ranks on its GPU), "policy": "rr" (the GPU's dispatcher takes one
    workgroup from each rank's launch in turn), "seq" (one rank's whole
    launch first) or "adv" (adversarial: a workgroup that will wait whenever
    some rank's next one does -- the dispatcher may pick any queue)}.  Each message is then `wgs`
    workgroups dispatched in the launch's message order (the kernel's
    blockIdx order); a dispatched workgroup holds its slot until its wait is
    satisfied; the message's flag moves when its last workgroup is done.  A
    residency stall is reported like a protocol deadlock, with
    "residency": True.  `stats` (if given) gets "max_launch_wgs" and
    "max_gpu_wgs" (the most workgroups of concurrent launches on one GPU)."""
    seq_s = [[0] * P for _ in range(P)]
    seq_r = [[0] * P for _ in range(P)]
    # ready[owner][from][slot], ack[owner][from][slot]: plain stores, as the
    # kernel does (a flag per pair would move backwards -- the bug this models)
    ready = [[[0] * SLOTS for _ in range(P)] for _ in range(P)]
    ack = [[[0] * SLOTS for _ in range(P)] for _ in range(P)]
    # per rank: list of ops (stream, deps, launches) over all calls
    ranks = []
    for r in range(P):
        ops, c_join, final_wait = pico_amd.schedule(coll, algo, P, r, count=count, rcounts=rcounts, esz=esz,
                                                    chunk_bytes=chunk_bytes, relay_min_bytes=relay_min_bytes,
                                                    trees=trees, flat_ag=flat_ag, flat_rs=flat_rs)
        seq = []
        base = 0
        host, hosted, defer = dm_tree_plan(ops, esz, slot) if dm_trees else ({}, {}, set())
        if stats is not None:
            stats.setdefault("deferred", 0)
            stats.setdefault("in_exchange", 0)
            stats["deferred"] += len(defer)
            stats["in_exchange"] += len(host) - len(defer)
        held = {}
        for _call in range(calls):
            # entries of this call with symbolic deps, resolved once every op
            # has its place (a tree may wait for a host issued after it)
            ents, at = [], {}
            first_c = None
            for i, o in enumerate(ops):
                stream = "C" if o["xchg"] else "K"
                deps = []
                if o["wait"] >= 0:
                    deps.append(("op", o["wait"]))
                launches = []
                if host.get(i) == i:
                    # a tree hosting itself: its own launch on the comm stream
                    # (after every K op issued before it), pulling its leaves
                    srcs = [x for x in defer if x < i and dm_tree_src(ops, x) == i]
                    launches = exchange_launches(r, [], [], seq_s[r], seq_r[r], slot, P, merge, held.pop(srcs[0]))
                    ents.append({"stream": "C", "deps": [("Kb-ent", len(ents))], "launches": launches})
                    # K takes up the tree's place: waits for that launch
                    stream, deps, launches = "K", [("ent", len(ents) - 1)], []
                elif i in host:
                    # the tree runs inside exchange host[i]: K waits for it there
                    stream, deps = "K", [("op", host[i])]
                elif o["xchg"]:
                    sends = [(p["peer"], p["count"] * esz, (p["src_buf"], p["src_off"])) for p in o["prims"]
                             if p["type"] == "SEND" and p["count"]]
                    recvs = [(p["peer"], p["count"] * esz) for p in o["prims"] if p["type"] == "RECV" and p["count"]]
                    if i in defer:
                        held[i] = recvs
                        recvs = []
                    dl = ()
                    if i in hosted:
                        j = hosted[i]
                        # a deferred tree: the leaves of the exchange that feeds it
                        srcs = [x for x in defer if x < i and dm_tree_src(ops, x) == j]
                        if srcs:
                            dl = held.pop(srcs[0])
                        # stream_join(C, K): the comm stream follows every K op issued so far
                        deps.append(("Kb-host", i, j))
                    launches = exchange_launches(r, sends, recvs, seq_s[r], seq_r[r], slot, P, merge, dl)
                    if first_c is None and c_join:
                        first_c = i
                        # c_join: the comm stream waits for the caller's stream's prior work
                        deps.append(("Kb-op", i))
                at[i] = len(ents)
                ents.append({"stream": stream, "deps": deps, "launches": launches})

            def res(d):
                if d[0] == "op":
                    return base + at[d[1]]
                if d[0] == "ent":
                    return base + d[1]
                if d[0] == "Kb-ent":
                    return ("K-before", base + d[1])
                if d[0] == "Kb-op":
                    return ("K-before", base + at[d[1]])
                return ("K-before-host", base + at[d[1]], base + at[d[2]])

            for e in ents:
                seq.append({"stream": e["stream"], "deps": [res(d) for d in e["deps"]], "launches": e["launches"],
                            "done": False, "li": 0, "started": False})
            if final_wait >= 0:
                # the caller's stream waits for the comm stream's op final_wait before the next call
                seq.append({"stream": "K", "deps": [base + at[final_wait]], "launches": [], "done": False, "li": 0,
                            "started": False})
            base = len(seq)
        ranks.append(seq)

    def dep_done(r, d):
        seq = ranks[r]
        if isinstance(d, tuple) and d[0] == "K-before-host":  # K ops issued before the host (not its tree)
            return all(seq[j]["done"] for j in range(d[1]) if seq[j]["stream"] == "K" and j != d[2])
        if isinstance(d, tuple):  # all K ops before index d
            return all(seq[j]["done"] for j in range(d[1]) if seq[j]["stream"] == "K")
        return seq[d]["done"]

    def head(r, stream):
        for j, op in enumerate(ranks[r]):
            if op["stream"] == stream and not op["done"]:
                return j
        return None

    res_on = residency is not None
    if res_on:
        gpu_of = residency["gpu_of"]
        ngpu = max(gpu_of) + 1
        free = [residency["slots"]] * ngpu
        share = [gpu_of.count(g) for g in range(ngpu)]
        policy = residency.get("policy", "rr")
        turn = [0] * ngpu

        def launch_wgs(r, launch):
            """the workgroups of each message of a launch (the library's cut applied if asked)"""
            if "wg" not in launch[0]:
                cw = [residency["wgs"]] * len(launch)
                if residency.get("cap"):
                    fit(cw, None, residency["slots"] // share[gpu_of[r]])
                for m, w in zip(launch, cw):
                    m["wg"], m["disp"], m["fin"] = w, 0, 0
                if stats is not None:
                    stats["max_launch_wgs"] = max(stats.get("max_launch_wgs", 0), sum(cw))
            return launch

    def cond(r, launch, m):
        """the flag condition of message m of rank r's current launch"""
        p, k = m["peer"], m["seq"] % SLOTS

        def ack_ok(x):
            return x["seq"] <= SLOTS or ack[r][x["peer"]][x["seq"] % SLOTS] >= x["seq"] - SLOTS

        if m["kind"] == "push":
            # a group writes only once every member's slot is free
            return ack_ok(m) and ("grp" not in m or all(ack_ok(x) for x in launch
                                                       if x["kind"] == "push" and x.get("grp") == m["grp"]))
        return ready[r][p][k] >= m["seq"]

    def complete(r, m):
        p, k = m["peer"], m["seq"] % SLOTS
        if m["kind"] == "push":
            assert ready[p][r][k] < m["seq"], "a ready flag would move backwards"
            ready[p][r][k] = m["seq"]
        else:
            assert ack[p][r][k] < m["seq"], "an ack flag would move backwards"
            ack[p][r][k] = m["seq"]
        m["done"] = True

    def current(r):
        """rank r's runnable comm-stream launch (deps met), or None"""
        j = head(r, "C")
        if j is None:
            return None
        op = ranks[r][j]
        if not all(dep_done(r, d) for d in op["deps"]) or op["li"] >= len(op["launches"]):
            return None
        return op["launches"][op["li"]]

    progress = True
    while progress:
        progress = False
        if res_on:
            # dispatch: each GPU fills its free slots from its ranks' current launches
            for g in range(ngpu):
                mine = [r for r in range(P) if gpu_of[r] == g]
                while free[g] > 0:
                    cands = []
                    for r in mine:
                        L = current(r)
                        if L is not None and any(m["disp"] < m["wg"] for m in launch_wgs(r, L)):
                            cands.append(r)
                    if not cands:
                        break
                    if policy == "seq":
                        r = cands[0]
                    elif policy == "adv":
                        # adversarial: a workgroup that will wait, if any rank's next one does
                        def nxt(x):
                            L = current(x)
                            return L, next(m for m in L if m["disp"] < m["wg"])
                        waiting = [x for x in cands if not cond(x, *nxt(x))]
                        r = (waiting or cands)[turn[g] % len(waiting or cands)]
                        turn[g] += 1
                    else:
                        r = cands[turn[g] % len(cands)]
                        turn[g] += 1
                    L = current(r)
                    m = next(x for x in L if x["disp"] < x["wg"])
                    m["disp"] += 1
                    free[g] -= 1
                    progress = True
                if stats is not None:
                    held = sum(m["disp"] - m["fin"] for r in mine for L in [current(r)] if L for m in L)
                    stats["max_gpu_wgs"] = max(stats.get("max_gpu_wgs", 0), held)
        for r in range(P):
            for stream in ("C", "K"):
                j = head(r, stream)
                if j is None:
                    continue
                op = ranks[r][j]
                if not all(dep_done(r, d) for d in op["deps"]):
                    continue
                if op["li"] >= len(op["launches"]):
                    op["done"] = True
                    progress = True
                    continue
                # the current launch: its messages progress independently
                launch = op["launches"][op["li"]]
                for m in launch:
                    if m.get("done"):
                        continue
                    if res_on:
                        # dispatched workgroups whose wait is over finish and free their slots
                        w = m["disp"] - m["fin"]
                        if w and cond(r, launch, m):
                            m["fin"] += w
                            free[gpu_of[r]] += w
                            progress = True
                            if m["fin"] == m["wg"]:
                                complete(r, m)
                        continue
                    if not cond(r, launch, m):
                        continue
                    complete(r, m)
                    progress = True
                if all(m.get("done") for m in launch):
                    op["li"] += 1
                    progress = True
    stuck = []
    for r in range(P):
        for stream in ("C", "K"):
            j = head(r, stream)
            if j is not None:
                op = ranks[r][j]
                pend = []
                if op["li"] < len(op["launches"]):
                    pend = [(m["kind"], m["peer"], m["seq"]) for m in op["launches"][op["li"]] if not m.get("done")]
                stuck.append((r, stream, j, op["deps"], pend))
    if not stuck:
        return None
    out = {"stuck": stuck, "ready": ready, "ack": ack}
    if res_on:
        out["residency"] = True
        out["free_slots"] = list(free)
    return out


def fit(cw, tw, cap):
    """restatement of dm_fit_residency (bine_internal.h; the library's own is
    tested against it through bine_dm_fit_residency): scale the parts
    proportionally, each >= 1, to sum <= cap; 0 unchanged, 1 scaled, -1 the
    parts alone exceed cap"""
    tot = sum(cw) + (tw[0] if tw else 0)
    parts = len(cw) + (1 if tw and tw[0] > 0 else 0)
    if cap <= 0 or tot <= cap:
        return 0
    if parts > cap:
        return -1
    for i in range(len(cw)):
        cw[i] = max(1, cw[i] * cap // tot)
    if tw and tw[0] > 0:
        tw[0] = max(1, tw[0] * cap // tot)
    s = sum(cw) + (tw[0] if tw else 0)
    while s > cap:
        if tw and tw[0] > 0 and tw[0] >= max(cw + [0]):
            tw[0] -= 1
        else:
            i = max(range(len(cw)), key=lambda x: (cw[x], -x))
            cw[i] -= 1
        s -= 1
    return 1


def fused_residency(P, W, slots, held=0, slices=True, order="rr"):
    """k_dm_fused's residency on ONE GPU shared by P ranks:
    each rank launches W workgroups; workgroup w does phase A (its pushes, no
    wait at a fresh slot), then waits for phase B's leaves, then for phase D's
    pieces, holding its slot until the end.  With slice flags (`slices`)
    workgroup w waits only for the peers' workgroup w; with whole-message
    flags for every workgroup of every peer.  The GPU has `slots` workgroup
    slots, `held` of them taken for the whole run by other waves; each rank's
    workgroups are dispatched in blockIdx order ("rr": one from each rank in
    turn, "seq": rank 0's launch first, ...).  Returns (completed, the most
    transport workgroups resident at once)."""
    state = [[0] * W for _ in range(P)]   # 0 not dispatched, 1 past A, 2 past B, 3 done
    nxt = [0] * P
    free = slots - held
    most = 0
    turn = 0

    def past(w, k):
        if slices:
            return all(state[r][w] >= k for r in range(P))
        return all(s >= k for row in state for s in row)

    progress = True
    while progress:
        progress = False
        while free > 0:
            cands = [r for r in range(P) if nxt[r] < W]
            if not cands:
                break
            r = cands[turn % len(cands)] if order == "rr" else cands[0]
            turn += 1
            state[r][nxt[r]] = 1
            nxt[r] += 1
            free -= 1
            progress = True
        most = max(most, sum(1 for row in state for s in row if s in (1, 2)))
        for r in range(P):
            for w in range(nxt[r]):
                if state[r][w] == 1 and past(w, 1):
                    state[r][w] = 2
                    progress = True
                if state[r][w] == 2 and past(w, 2):
                    state[r][w] = 3
                    free += 1
                    progress = True
    return all(s == 3 for row in state for s in row), most
