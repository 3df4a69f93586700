"""Position-level simulation of the fsm16 kernel's z-block stream (analysis
tool, not product): replays the per-sweep change record of tools/sched/
record.py under admission policies and counts stream positions.

Every policy is checked for exactness: a block that changes in a sweep must
be visited in it (asserted).  Timing model (fsm16_kernel.hip, fsm_common.h):
one position = kb steps; a visit is in flight (its change unknown) for infl
positions; a block's visit is >= vis positions after its upwind x/y (and, for
a run restarted in the same tile, z) neighbour's visit.

Policies
  cur   the kernel's rule (decide16): block changed at its last visit, a face
        neighbour changed since, or the sweep-upwind x/y neighbour in flight;
        a tile's run goes from its first such block to the column end.
  face  as cur, but a neighbour counts only if it changed the face layer it
        shares with the block (settled visits only).
  hold  per-tile frontiers: a block is decided when its upwind x/y blocks
        and its z-below are decided; with a settled reason it is visited,
        with an in-flight dependency it waits (the tile is held), otherwise
        it is skipped.  When no block is ready the stream fills the position
        with the oldest held block (hold) or a bubble (holdb).
  hold+face, holdb+face  the two combined.
"""
import argparse
import sys
from collections import deque

import numpy as np

SWEEPS = [(0, 0, 0), (1, 0, 0), (0, 1, 0), (1, 1, 0), (0, 0, 1), (1, 0, 1), (0, 1, 1), (1, 1, 1)]


def diag_order(ntx, nty):
    ids = [(tx, ty) for ty in range(nty) for tx in range(ntx)]
    ids.sort(key=lambda t: (t[0] + t[1], t[1]))
    return ids


class Geo:
    def __init__(self, nx, ny, nz, zb=32):
        self.ntx, self.nty, self.nzk = -(-nx // 8), -(-ny // 8), -(-nz // zb)
        self.nt = self.ntx * self.nty
        self.nb = self.nt * self.nzk
        self.order = diag_order(self.ntx, self.nty)

    def bid(self, tx, ty, tz):
        return tz * self.nt + ty * self.ntx + tx


FACE_OPP = [1, 0, 3, 2, 5, 4]


def neighbours(g, b):
    """[(face of b, neighbour block)] for the existing face neighbours."""
    tz, r = divmod(b, g.nt)
    ty, tx = divmod(r, g.ntx)
    out = []
    if tx > 0: out.append((0, b - 1))
    if tx < g.ntx - 1: out.append((1, b + 1))
    if ty > 0: out.append((2, b - g.ntx))
    if ty < g.nty - 1: out.append((3, b + g.ntx))
    if tz > 0: out.append((4, b - g.nt))
    if tz < g.nzk - 1: out.append((5, b + g.nt))
    return out


class State:
    def __init__(self, g, bc, face_rule):
        self.g = g
        self.lp = np.full(g.nb, 2, np.int64)
        self.chg = np.full(g.nb, 1, np.int64)
        self.chg[bc] = 3
        # fchg[b, f]: clock of b's last visit that changed its face f (BC blocks: every face)
        self.fchg = np.full((g.nb, 6), 1, np.int64)
        self.fchg[bc] = 3
        self.face_rule = face_rule
        self.nbr = [neighbours(g, b) for b in range(g.nb)]
        self.pending = deque()          # (settle clock, block, changed, faces)

    def settle(self, C):
        while self.pending and self.pending[0][0] <= C:
            _, b, c, f, clk = self.pending.popleft()
            if c:
                self.chg[b] = clk
            self.fchg[b, f] = clk             # (faces change only with the block)

    def reason(self, b):
        lp = self.lp[b]
        if self.chg[b] >= lp:
            return 1
        for fb, nb in self.nbr[b]:
            if self.face_rule:
                if self.fchg[nb, FACE_OPP[fb]] > lp:
                    return 2
            elif self.chg[nb] > lp:
                return 2
        return 0


CONT = False
PAR = False
LEVEL = False
FORCEK = None


def run(rec_chg, rec_face, bc, g, policy, kb=2, infl=9, vis=6, rel=None):
    """rel: (own_rel, face_rel) of record.py --rel: the marks a visit leaves
    for later decisions (its own revisit, its face neighbours) follow the
    relevance rule instead of every change; exactness is still asserted
    against the actual changes."""
    face_rule = policy.endswith("+face") or policy == "face"
    base = "cur" if policy == "face" else policy.replace("+face", "")
    S = State(g, bc, face_rule)
    clock = 64
    tot = dict(pos=0, visits=0, bubbles=0, forced=0, steps=0, checks=0, cont=0, rounds=0, zstart=0, zend=0)
    why = np.zeros(5, np.int64)                  # visits by reason: 1 self 2 neighbour 3 inflight 4 run/forced
    why_chg = np.zeros(5, np.int64)
    nsweep = len(rec_chg)
    for s in range(nsweep):
        rx, ry, rz = SWEEPS[s % 8]
        chg_s, face_s = rec_chg[s], rec_face[s]
        mark_s, mface_s = (chg_s, face_s) if rel is None else (rel[0][s], rel[1][s])
        visited = np.zeros(g.nb, bool)
        last_admit = [None]
        zorder = list(range(g.nzk))[::-1] if rz else list(range(g.nzk))
        tiles = [((g.ntx - 1 - tx) if rx else tx, (g.nty - 1 - ty) if ry else ty) for tx, ty in g.order]
        tindex = {t: i for i, t in enumerate(tiles)}

        def up(t, dx, dy):
            tx, ty = t
            if dx:
                ux = tx + (1 if rx else -1)
                return (ux, ty) if 0 <= ux < g.ntx else None
            uy = ty + (1 if ry else -1)
            return (tx, uy) if 0 <= uy < g.nty else None

        def admit(b, C, r):
            # z-boundary values from HBM: a run start above the column's first
            # block (z-upwind node) / a run end below its last (z-downwind node)
            tz = b // g.nt
            k = zorder.index(tz)
            zb_ = g.bid(*divmod(b % g.nt, g.ntx)[::-1], zorder[k - 1]) if k > 0 else None
            if zb_ is not None and S.lp[zb_] != C - 1:
                tot["zstart"] += 1
            if last_admit[0] is not None:
                pb, pk = last_admit[0]
                if pk < g.nzk - 1 and not (b == g.bid(*divmod(pb % g.nt, g.ntx)[::-1], zorder[pk + 1])):
                    tot["zend"] += 1
            last_admit[0] = (b, k)
            visited[b] = True
            S.lp[b] = C
            c = bool(chg_s[b])
            S.pending.append((C + infl, b, bool(mark_s[b]), mface_s[b].copy(), C))
            why[r] += 1
            why_chg[r] += c
            tot["visits"] += 1

        C = clock
        if base == "cur":
            for t in tiles:
                S.settle(C) if face_rule else None
                # decisions for this tile happen now: first kz with a reason
                k0 = None
                rs = []
                for k in range(g.nzk):
                    tz = zorder[k]
                    b = g.bid(t[0], t[1], tz)
                    if not face_rule:
                        S.settle(C)
                    r = S.reason(b)
                    if not r:
                        for dx, dy in ((1, 0), (0, 1)):
                            u = up(t, dx, dy)
                            if u is not None and S.lp[g.bid(u[0], u[1], tz)] > C - infl:
                                r = 3
                    rs.append(r)
                    if r and k0 is None:
                        k0 = k
                if k0 is None:
                    continue
                need = 0
                for k in range(k0, g.nzk):
                    tz = zorder[k]
                    p = -10 ** 9
                    for dx, dy in ((1, 0), (0, 1)):
                        u = up(t, dx, dy)
                        if u is not None:
                            p = max(p, S.lp[g.bid(u[0], u[1], tz)])
                    need = max(need, p + vis - (k - k0) - C)
                C += need
                tot["bubbles"] += need
                for k in range(k0, g.nzk):
                    S.settle(C)
                    b = g.bid(t[0], t[1], zorder[k])
                    r = S.reason(b)
                    if not r:
                        r = 3 if rs[k] == 3 else 4
                    admit(b, C, r)
                    C += 1
        elif PAR:
            # the kernel's form: fast path = the current tile's next block; else
            # windows of 64 tiles (diagonal order from the first incomplete tile),
            # every lane one decision per round on a snapshot of the frontiers
            fz = {t: 0 for t in tiles}
            done = 0
            last_t = None

            def status(t):
                k = fz[t]
                if k == g.nzk:
                    return "done", None, 0
                tz = zorder[k]
                ups = [up(t, 1, 0), up(t, 0, 1)]
                if any(u is not None and fz[u] <= k for u in ups):
                    return "blocked", None, 0
                b = g.bid(t[0], t[1], tz)
                deps = [g.bid(u[0], u[1], tz) for u in ups if u is not None]
                zb = g.bid(t[0], t[1], zorder[k - 1]) if k > 0 else None
                run_on = zb is not None and S.lp[zb] == C - 1
                dep_lp = [S.lp[d] for d in deps] + ([S.lp[zb]] if zb is not None and not run_on else [])
                r = S.reason(b)
                if r:
                    return ("ready" if all(l + vis <= C for l in dep_lp) else "wait"), b, r
                if any(l > C - infl for l in dep_lp) or run_on:
                    return "held", b, 0
                return "skip", b, 0

            nbub = 0
            while done < len(tiles):
                S.settle(C)
                chosen = None
                heldc = None
                if last_t is not None:
                    st_, b, r = status(last_t)
                    tot["checks"] += 1
                    if st_ == "ready":
                        chosen = (last_t, b, r)
                        tot["cont"] += 1
                if chosen is None:
                    while done < len(tiles) and fz[tiles[done]] == g.nzk:
                        done += 1
                    base = done
                    while chosen is None and base < len(tiles):
                        win = tiles[base:base + 64]
                        while True:
                            tot["rounds"] += 1
                            sts = [status(t) for t in win]
                            if heldc is None:
                                for i, x in enumerate(sts):
                                    if x[0] == "held":
                                        heldc = (win[i], x[1])
                                        break
                            rdy = [i for i, x in enumerate(sts) if x[0] == "ready"]
                            if LEVEL and rdy:
                                # the ready block on the lowest hyperplane diag + k first
                                rdy.sort(key=lambda i: (tindex[win[i]] and (win[i][0] if not rx else g.ntx - 1 - win[i][0])
                                                        + (win[i][1] if not ry else g.nty - 1 - win[i][1])) + fz[win[i]])
                            skips = [i for i, x in enumerate(sts) if x[0] == "skip"]
                            for i in skips:
                                fz[win[i]] += 1
                            if rdy:
                                i = rdy[0]
                                chosen = (win[i], sts[i][1], sts[i][2])
                                break
                            if not skips:
                                break
                        base += 64
                while done < len(tiles) and fz[tiles[done]] == g.nzk:
                    done += 1
                if chosen is None and FORCEK is not None and heldc is not None and nbub >= FORCEK:
                    t, b = heldc
                    # forced: visible only if its upwind visits are >= vis back
                    tz = b // g.nt
                    ok = True
                    for dx, dy in ((1, 0), (0, 1)):
                        u = up(t, dx, dy)
                        if u is not None and S.lp[g.bid(u[0], u[1], tz)] + vis > C:
                            ok = False
                    k_ = zorder.index(tz)
                    if k_ > 0:
                        zb_ = g.bid(t[0], t[1], zorder[k_ - 1])
                        if S.lp[zb_] != C - 1 and S.lp[zb_] + vis > C:
                            ok = False
                    if ok:
                        chosen = (t, b, 4)
                        tot["forced"] += 1
                if chosen is None:
                    if done >= len(tiles):
                        break
                    tot["bubbles"] += 1
                    nbub += 1
                    C += 1
                    continue
                nbub = 0
                t, b, r = chosen
                admit(b, C, r)
                last_t = t
                fz[t] += 1
                C += 1
        else:
            fz = {t: 0 for t in tiles}
            left = len(tiles)
            last_t = None
            while left:
                S.settle(C)
                chosen = None
                held = None
                scan = tiles
                if CONT and last_t is not None and fz[last_t] < g.nzk:
                    scan = [last_t] + [t for t in tiles if t != last_t]
                for t in scan:
                    while fz[t] < g.nzk:
                        k = fz[t]
                        tz = zorder[k]
                        ups = [up(t, 1, 0), up(t, 0, 1)]
                        if any(u is not None and fz[u] <= k for u in ups):
                            break                                     # upwind undecided
                        b = g.bid(t[0], t[1], tz)
                        deps = [g.bid(u[0], u[1], tz) for u in ups if u is not None]
                        zb = g.bid(t[0], t[1], zorder[k - 1]) if k > 0 else None
                        r = S.reason(b)
                        tot["checks"] += 1
                        # z-below admitted at the previous position: a run continues in registers
                        run_on = zb is not None and S.lp[zb] == C - 1
                        dep_lp = [S.lp[d] for d in deps] + ([S.lp[zb]] if zb is not None and not run_on else [])
                        if r:
                            if all(l + vis <= C for l in dep_lp):
                                chosen = (t, b, r)
                            elif held is None:
                                held = ("vis", t, b)
                            break
                        if any(l > C - infl for l in dep_lp) or run_on:
                            if held is None and all(l + vis <= C for l in dep_lp):
                                held = ("inf", t, b)
                            break
                        fz[t] += 1                                    # skip (free)
                        if fz[t] == g.nzk:
                            left -= 1
                    if chosen:
                        break
                if chosen:
                    t, b, r = chosen
                    admit(b, C, r)
                    tot["cont"] += t == last_t
                    last_t = t
                elif base == "hold" and held is not None and held[0] == "inf":
                    _, t, b = held
                    admit(b, C, 4)
                    tot["forced"] += 1
                elif left:
                    tot["bubbles"] += 1
                    C += 1
                    continue
                else:
                    break
                fz[t] += 1
                if fz[t] == g.nzk:
                    left -= 1
                C += 1
        missed = np.flatnonzero(chg_s & ~visited)
        assert len(missed) == 0, (policy, s, missed[:8])
        n = C - clock
        tot["pos"] += n
        tot["steps"] += n * kb + 16 if n else 0
        clock = C + infl
    S.settle(clock + 10 ** 9)
    tot["why"] = why[1:].tolist()
    tot["why_chg"] = why_chg[1:].tolist()
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("rec")
    ap.add_argument("--policies", default="cur,face,hold,holdb,hold+face,holdb+face")
    ap.add_argument("--cont", action="store_true", help="hold policies: the current run's next block first")
    ap.add_argument("--par", action="store_true", help="hold policies: the kernel's parallel scan (holdb only)")
    ap.add_argument("--kb", type=int, default=2, help="steps per position (fsm16: 2; the 8-z kernel: 4)")
    ap.add_argument("--rel", action="store_true", help="marks by the relevance rule (record.py --rel)")
    ap.add_argument("--infl", type=int, default=0, help="positions a visit stays in flight (0: the kernel's 1 + ceil(16 / kb))")
    ap.add_argument("--level", action="store_true", help="--par: the ready block of the lowest diag + k first")
    ap.add_argument("--forcek", type=int, default=None, help="--par: after k bubbles in a row visit a held block")
    a = ap.parse_args()
    global CONT, PAR, LEVEL, FORCEK
    CONT = a.cont
    PAR = a.par
    LEVEL = a.level
    FORCEK = a.forcek
    R = np.load(a.rec)
    g = Geo(int(R["nx"]), int(R["ny"]), int(R["nz"]), zb=int(R["zb"]) if "zb" in R else 32)
    nst = len(R["stations"])
    agg = {}
    for pol in a.policies.split(","):
        acc = None
        for k in range(nst):
            ah = 2
            t = run(R[f"chg{k}"], R[f"face{k}"], R[f"bc{k}"], g, pol, kb=a.kb,
                    infl=a.infl or 1 + -(-(14 + ah) // a.kb),
                    vis=-(-12 // a.kb), rel=(R[f"own_rel{k}"], R[f"face_rel{k}"]) if a.rel else None)
            acc = t if acc is None else {key: (acc[key] + t[key] if not isinstance(t[key], list)
                                               else [x + y for x, y in zip(acc[key], t[key])]) for key in t}
        agg[pol] = acc
        base = agg.get("cur", acc)
        print(f"{pol:12s} positions/solve {acc['pos'] / nst:9.1f}  steps {acc['steps'] / nst:9.1f} "
              f"({acc['steps'] / base['steps']:.3f} of cur)  visits {acc['visits'] / nst:8.1f}  bubbles "
              f"{acc['bubbles'] / nst:7.1f}  forced {acc['forced'] / nst:6.1f}  checks/pos {acc['checks'] / max(1, acc['pos']):.1f} rounds/pos {acc['rounds'] / max(1, acc['pos']):.2f} zstart {acc['zstart'] / nst:.0f} zend {acc['zend'] / nst:.0f} cont {acc['cont'] / nst:.0f}  by reason (self, nbr, inflight, run) "
              f"{[round(x / nst) for x in acc['why']]} changed {[round(x / nst) for x in acc['why_chg']]}", flush=True)


if __name__ == "__main__":
    sys.exit(main())
