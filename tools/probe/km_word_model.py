"""CPU model of kmeans.hip's word-scan cluster-0 sum (km_word_sum): the
cumulative cluster-0 sum of KMeans::Run (kmldpc/src/kmeans.cc:33-46: idxSum[0]
+= data_[j] in ascending j, cumulative over iterations) computed per 64-symbol
WORD instead of per element, with per-word summaries cached across iterations.

While the running sum acc stays in one binade [2^(e-1), 2^e) (sign sg), every
rounded add is a move on the grid u = 2^(e-53): with A = |acc| / u and
X = sg x / u, RN(acc + x) = sg (A + rint(X)) u unless X is a tie (frac 0.5:
the parity of the corrected prefix decides, ties to even) or the result leaves
the binade.  A word's summary at (e, sg) — its members' grid sum G, the min
and max of its local prefixes, its ties' local prefix parities — depends only
on (membership mask, e, sg), so it is cached per word and recomputed only when
one of those changes.  An exclusive scan of the G over the words gives every
word's starting prefix; the first word whose prefixes may leave
[2^52 + margin, 2^53 - margin] (or that holds a large element / too many ties)
is added element by element with real fp64 adds, and the scan resumes after it
at the new binade.  Ties are resolved in order afterwards from the parities.

This model replays those steps with Python doubles (the DPP scan's tree order
included) and checks them against the plain left-to-right sum on random,
sign-changing, tie-heavy and extreme inputs, over many iterations with slowly
changing membership (cache hits) like the real k-means.
Run: python tools/probe/km_word_model.py"""
import math
import random
import sys

MARGIN = 64.0
MAX_TIES = 32
LO, HI = 2.0 ** 52 + MARGIN, 2.0 ** 53 - MARGIN


def seq_sum(acc, xs):
    for x in xs:
        acc = acc + x
    return acc


def rint(x):
    return float(round(x)) if math.isfinite(x) else x


def frexp_exp(x):
    return math.frexp(x)[1]


def scan_ok(acc):
    return math.isfinite(acc) and abs(acc) >= 2.0 ** -960 and acc != 0.0


def parity(v):  # v an integer-valued double
    if not math.isfinite(v):
        return 0
    h = v * 0.5
    return 1 if h != math.floor(h) else 0


def walk(vals, e, sg):
    """summary of one word's members (ascending) at binade e, sign sg"""
    P = 0.0
    mn, mx = math.inf, -math.inf
    ntie, tpar, hard = 0, 0, False
    for x in vals:
        X = math.ldexp(sg * x, 53 - e) if math.isfinite(x) else x
        big = not (abs(X) < 2.0 ** 51)
        if big:  # the word is added element by element; its summary is unused
            hard = True
            continue
        fl = math.floor(X)
        tie = (X - fl) == 0.5
        P = P + (fl if tie else rint(X))
        if tie:
            if ntie < MAX_TIES:
                tpar |= parity(P) << ntie
            ntie += 1
        mn = min(mn, P)
        mx = max(mx, P)
    if ntie > MAX_TIES:
        hard = True
    return dict(G=P, mn=mn, mx=mx, ntie=ntie, tpar=tpar, hard=hard)


def dpp_exclusive_scan(g):
    """the kernel's exclusive scan over <= 32 lanes: shift by one lane, then
    row_shr 1/2/4/8 inside rows of 16 and row_bcast:15 into the second row
    (the same association order as the hardware)"""
    n = 32
    v = [0.0] + [g[i - 1] if i - 1 < len(g) else 0.0 for i in range(1, n)]
    for s in (1, 2, 4, 8):
        v = [v[i] + v[i - s] if (i % 16) >= s else v[i] for i in range(n)]
    v = [v[i] + v[15] if i >= 16 else v[i] for i in range(n)]
    return v


class Chain:
    def __init__(self, nwords):
        self.cache = [None] * nwords  # (key, summary)
        self.walks = 0
        self.rounds = 0
        self.seq = 0


def word_sum(acc, words, masks, chain):
    """acc + the members of every word (masks[w]: their values words[w]) in
    ascending order, the sequential rounding, by the word-scan method"""
    Sw = len(words)
    w0 = 0
    while w0 < Sw:
        chain.rounds += 1
        if not scan_ok(acc):
            for x in words[w0]:
                acc = acc + x
            chain.seq += len(words[w0])
            w0 += 1
            continue
        e = frexp_exp(acc)
        sg = -1.0 if acc < 0.0 else 1.0
        A = math.ldexp(abs(acc), 53 - e)
        summ = []
        for w in range(Sw):
            if w < w0:
                summ.append(None)
                continue
            key = (masks[w], e, sg)
            c = chain.cache[w]
            if c is None or c[0] != key:
                chain.walks += 1
                c = (key, walk(words[w], e, sg))
                chain.cache[w] = c
            summ.append(c[1])
        g = [summ[w]["G"] if w >= w0 else 0.0 for w in range(Sw)]
        E = dpp_exclusive_scan(g)
        wf = Sw
        for w in range(w0, Sw):
            s = summ[w]
            if s["hard"] or A + E[w] + s["mn"] < LO or A + E[w] + s["mx"] > HI:
                wf = w
                break
        # too many ties before wf: the word where the running count passes MAX_TIES fails
        nt = 0
        for w in range(w0, wf):
            nt += summ[w]["ntie"]
            if nt > MAX_TIES:
                wf = w
                break
        U = 0
        for w in range(w0, wf):
            s = summ[w]
            q0 = parity(A + E[w])
            for i in range(s["ntie"]):
                r = q0 ^ ((s["tpar"] >> i) & 1) ^ (U & 1)
                U += r
        T = A + E[wf] + U if wf < 32 else None
        if wf == Sw:
            T = A + (E[Sw - 1] + g[Sw - 1]) + U if Sw > 0 else A
        acc = sg * math.ldexp(T, e - 53)
        if wf == Sw:
            break
        for x in words[wf]:
            acc = acc + x
        chain.seq += len(words[wf])
        w0 = wf + 1
    return acc


def kmeans_like(rng, nwords=18, iters=20, kind="qpsk"):
    """a stream of iterations: symbols fixed, membership drifting slowly"""
    S = 64 * nwords
    if kind == "qpsk":
        c = complex(rng.gauss(0, 0.7), rng.gauss(0, 0.7))
        ys = [c + complex(rng.gauss(0, 0.5), rng.gauss(0, 0.5)) for _ in range(S)]
        vals = [y.real for y in ys]
    elif kind == "ties":  # values on a coarse grid: ties everywhere
        vals = [rng.randint(-64, 400) * 2.0 ** rng.randint(-6, 1) for _ in range(S)]
    elif kind == "signs":  # a cluster centre near the axis: mixed signs
        vals = [rng.gauss(0.02, 0.5) for _ in range(S)]
    elif kind == "extreme":
        vals = [rng.choice([1.0, -1.0]) * 2.0 ** rng.uniform(-60, 30) for _ in range(S)]
    elif kind == "bigsmall":
        vals = [rng.gauss(0, 1) * (1e6 if rng.random() < 0.01 else 1.0) for _ in range(S)]
    else:
        raise ValueError(kind)
    member = [rng.random() < 0.25 for _ in range(S)]
    return vals, member


def run(seed, kind, nwords=18, iters=20):
    rng = random.Random(seed)
    vals, member = kmeans_like(rng, nwords, iters, kind)
    ch = Chain(nwords)
    acc_ref = acc = 0.0
    for it in range(iters):
        if it > 0:  # a few membership flips per iteration, fewer later
            for _ in range(rng.randint(0, max(0, 6 - it // 3))):
                j = rng.randrange(len(vals))
                member[j] = not member[j]
        words, masks = [], []
        for w in range(nwords):
            m = 0
            xs = []
            for b in range(64):
                if member[64 * w + b]:
                    m |= 1 << b
                    xs.append(vals[64 * w + b])
            words.append(xs)
            masks.append(m)
        flat = [x for xs in words for x in xs]
        acc_ref = seq_sum(acc_ref, flat)
        acc = word_sum(acc, words, masks, ch)
        if not (acc == acc_ref or (math.isnan(acc) and math.isnan(acc_ref))):
            return False, (it, acc, acc_ref), ch
        if acc == acc_ref and acc == 0.0 and math.copysign(1, acc) != math.copysign(1, acc_ref):
            return False, (it, "signed zero"), ch
    return True, None, ch


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    tot = {"walks": 0, "rounds": 0, "seq": 0, "runs": 0}
    for kind in ("qpsk", "ties", "signs", "extreme", "bigsmall"):
        for s in range(n):
            ok, why, ch = run(1000 * s + 7, kind)
            if not ok:
                print("MISMATCH", kind, s, why)
                sys.exit(1)
            if kind == "qpsk":
                tot["walks"] += ch.walks
                tot["rounds"] += ch.rounds
                tot["seq"] += ch.seq
                tot["runs"] += 1
        print(f"{kind}: {n} streams x 20 iterations exact")
    r = tot["runs"] * 20
    print(f"qpsk: per iteration {tot['walks'] / r:.2f} word walks, {tot['rounds'] / r:.2f} scan rounds, "
          f"{tot['seq'] / r:.1f} elements added one by one")


if __name__ == "__main__":
    main()
