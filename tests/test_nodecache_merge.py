"""The lemma behind nc_group_kernel (opendht_amd/csrc/kad_engine.hip): NodeCache::getCachedNodes'
two-pointer walk (node_cache.cpp:36-66) is a greedy merge of the left and right runs, and in a greedy
merge of two sequences with distinct values an element's place is its index plus the number of
elements of the other sequence whose prefix maximum is below its own prefix maximum."""
import random


def _greedy(A, B):
    i = j = 0
    out = []
    while i < len(A) or j < len(B):
        if i == len(A) or (j < len(B) and not A[i] < B[j]):
            out.append(("b", j))
            j += 1
        else:
            out.append(("a", i))
            i += 1
    return out


def _by_prefix_max(A, B):
    Am = [max(A[:i + 1]) for i in range(len(A))]
    Bm = [max(B[:j + 1]) for j in range(len(B))]
    pos = {("a", i): i + sum(b < Am[i] for b in Bm) for i in range(len(A))}
    pos.update({("b", j): j + sum(a < Bm[j] for a in Am) for j in range(len(B))})
    return sorted(pos, key=pos.get), sorted(pos.values())


def test_greedy_merge_prefix_max_lemma():
    rnd = random.Random(5)
    for _ in range(20000):
        vals = rnd.sample(range(1000), rnd.randint(0, 24))
        k = rnd.randint(0, len(vals))
        order, places = _by_prefix_max(vals[:k], vals[k:])
        assert order == _greedy(vals[:k], vals[k:])
        assert places == list(range(len(vals)))


def _walk_window(keys, exp, p, t, count):
    """NodeCache::getCachedNodes' two-pointer walk (node_cache.cpp:36-66) over a window of sorted keys with lb = p,
    stopped at the window's ends: the non-expired positions it emits, and whether it ran off an end of the window."""
    out, l, r = [], p - 1, p
    while len(out) < count and (l >= 0 or r < len(keys)):
        if l < 0:
            e, r = r, r + 1
        elif r >= len(keys):
            e, l = l, l - 1
        elif (keys[l] ^ t) < (keys[r] ^ t):
            e, l = l, l - 1
        else:
            e, r = r, r + 1
        if not exp[e]:
            out.append(e)
    return out


def _lane_answer(keys, exp, p, t, count, trunc_left, trunc_right, steps=24):
    """ncl2_lane_answer's algorithm (kad_engine.hip) on one line, in integers: keys as (run max << 8 | side << 7 |
    tie-break << 1 | expired) with the tie-break 63 - e on the left and e on the right, the 37 keys followed by NONE
    as a bitonic sequence of 64 (no shift by p), one half-cleaner at h = 32, then the first `steps` sorted (24: the
    kernel's KAD_NCL2_STEPS; 32: five levels of 16 compare-exchanges), then the first `count` non-expired keys up to
    the smaller end key of a truncated side. Returns the positions it
    emits, or None where the kernel sends the query to the wave path."""
    NONE, S = 0xFFFFFFFF, len(keys)
    d = [((k ^ t) << 8) | e for k, e in zip(keys, exp)]
    k = list(d)
    run = 0
    for e in range(p - 1, -1, -1):
        run = max(run, d[e] & ~255)
        k[e] = run | ((63 - e) << 1) | (d[e] & 1)
    run = 0
    for e in range(p, S):
        run = max(run, d[e] & ~255)
        k[e] = run | 128 | (e << 1) | (d[e] & 1)
    lim = min(k[0] | 1 if trunc_left else NONE, k[S - 1] | 1 if trunc_right else NONE)
    seq = k + [NONE] * (64 - S)
    # the sequence is bitonic: descending over the left run, ascending over the right run, then NONE
    w = [min(seq[r], seq[r + 32]) for r in range(32)]

    def clean(lo, n, h):  # half-cleaners h, h/2, .., 1 over w[lo:lo+n]
        while h:
            for r in range(lo, lo + n):
                if (r - lo) & h == 0 and w[r] > w[r + h]:
                    w[r], w[r + h] = w[r + h], w[r]
            h //= 2

    if steps == 32:
        clean(0, 32, 16)
    else:  # KAD_NCL2_STEPS = 24: the 16 smallest sorted, then the smaller half of the upper 16 sorted
        for r in range(16):
            if w[r] > w[r + 16]:
                w[r], w[r + 16] = w[r + 16], w[r]
        clean(0, 16, 8)
        for r in range(16, 24):
            w[r] = min(w[r], w[r + 8])
        clean(16, 8, 4)
        w = w[:24]
    assert w == sorted(k)[:steps]
    keep = [x for x in w if x <= lim and not x & 1]
    if len(keep) < count and (lim != NONE or w[steps - 1] != NONE):
        return None
    return [(x >> 1) & 63 if x & 128 else 63 - ((x >> 1) & 63) for x in keep[:count]]


def test_lane_answer_is_the_walk():
    """The count <= 14 NodeCache lane kernel's walk (bitonic merge of the two runs by run maximum, no window shift)
    equals the reference's two-pointer walk wherever it answers, and sends a query to the wave path only when the
    walk may leave the line."""
    rnd = random.Random(11)
    answered = 0
    for _ in range(4000):
        S = 37
        keys = sorted(rnd.sample(range(1 << 24), S))
        exp = [rnd.random() < 0.12 for _ in range(S)]
        p = rnd.randint(11, 26)
        t = rnd.randint(keys[p - 1] + 1, keys[p]) if keys[p] > keys[p - 1] + 1 else keys[p]
        count = rnd.randint(1, 14)
        tl, tr = rnd.random() < 0.8, rnd.random() < 0.8
        got = _lane_answer(keys, exp, p, t, count, tl, tr, steps=rnd.choice((24, 32)))
        walk = _walk_window(keys, exp, p, t, count)
        if got is None:
            continue
        answered += 1
        assert got == walk
        # an answer the kernel trusts never depends on nodes beyond a truncated end of the line: the same walk over
        # the line with up to 16 more sorted nodes past each truncated end (any keys, any expired flags)
        nl = rnd.randint(1, 16) if tl else 0
        nr = rnd.randint(1, 16) if tr else 0
        left = sorted(rnd.sample(range(keys[0]), min(nl, keys[0]))) if nl else []
        right = sorted(rnd.sample(range(keys[-1] + 1, 1 << 25), nr)) if nr else []
        wide = _walk_window(left + keys + right, [rnd.random() < 0.5 for _ in left] + exp +
                            [rnd.random() < 0.5 for _ in right], p + len(left), t, count)
        assert [e - len(left) for e in wide] == got
    assert answered > 3000


def test_search_insert_without_bad_nodes_is_order_free():
    """The premise of the swarm's all-online merge network (kad_swarm.hip, merge_lookup_net): without bad nodes,
    Search::insertNode (dht.cpp:961-1047: a node already in the list is skipped, an insert beyond a full list of
    SEARCH_NODES is refused, a list over SEARCH_NODES drops its farthest) keeps exactly the SEARCH_NODES closest of
    the list and everything inserted, whatever the order of the inserts, each node with the flags it had."""
    SN = 14
    rnd = random.Random(17)
    for _ in range(3000):
        pool = rnd.sample(range(10 ** 6), 60)
        start = sorted(rnd.sample(pool, rnd.randint(0, SN)))
        flags = {x: rnd.random() < 0.5 for x in start}
        answers = [rnd.choice(pool) for _ in range(rnd.randint(0, 32))]
        lst = list(start)
        for a in answers:  # sequential inserts (distance = the value itself)
            if a in lst:
                continue
            pos = sum(x < a for x in lst)
            if len(lst) >= SN and pos >= len(lst):
                continue
            lst.insert(pos, a)
            if len(lst) > SN:
                lst.pop()
        want = sorted(set(start) | set(answers))[:SN]
        assert lst == want
        assert [flags.get(x, False) for x in lst] == [flags.get(x, False) for x in want]


def _cx(k, i, a, b):
    if k[b] < k[a]:
        k[a], k[b] = k[b], k[a]
        i[a], i[b] = i[b], i[a]


_SORT8 = [(0, 1), (2, 3), (4, 5), (6, 7), (0, 2), (1, 3), (4, 6), (5, 7), (1, 2), (5, 6), (0, 4), (1, 5), (2, 6),
          (3, 7), (2, 4), (3, 5), (1, 2), (3, 4), (5, 6)]


def _closest_net(levels, K=8):
    """kad_swarm.hip peer_closest<8, true> restated: each bucket's slots (64-bit distance, node) sorted by the 19
    compare-exchanges, merged into the running top 8 by a half-cleaner against the bucket reversed and three levels;
    None (TIE) where the top 8 holds two equal distances or its last equals the nearest node left out."""
    MAX = (1 << 64) - 1
    L0, LI, nin, nl = None, None, MAX, 0
    for lv in levels:
        bk = [d for d, _ in lv] + [MAX] * (K - len(lv))
        bi = [n for _, n in lv] + [None] * (K - len(lv))
        if any(d == MAX for d, _ in lv):
            return None
        for a, b in _SORT8:
            _cx(bk, bi, a, b)
        if L0 is None:
            L0, LI = bk, bi
        else:
            for s in range(K):
                sw = bk[K - 1 - s] < L0[s]
                nin = min(nin, L0[s] if sw else bk[K - 1 - s])
                if sw:
                    L0[s], LI[s] = bk[K - 1 - s], bi[K - 1 - s]
            h = K // 2
            while h >= 1:
                for r in range(K):
                    if r & h == 0:
                        _cx(L0, LI, r, r + h)
                h //= 2
        nl = min(nl + len(lv), K)
    if any(L0[s] != MAX and L0[s] == L0[s + 1] for s in range(K - 1)) or (nin != MAX and L0[K - 1] == nin):
        return None
    return LI[:nl]


def test_query_network_is_the_inserts():
    """The swarm query kernel's sorting-network findClosestNodes (kad_swarm.hip peer_closest<8, true>) returns the
    routing_table.cpp:79-110 result (the window's nodes ranked by the full XOR distance: here the 64-bit top, then
    the tail) wherever it does not return TIE, and returns TIE only where 64-bit distances are equal; distances are
    drawn from a small range so that ties are common."""
    rnd = random.Random(23)
    seen_tie = seen_ok = 0
    for _ in range(4000):
        span = rnd.choice([40, 1000, 1 << 64])
        nodes = iter(range(10 ** 6))
        levels = [[(rnd.randrange(span), next(nodes)) for _ in range(rnd.randint(1 if j == 0 else 0, 8))]
                  for j in range(rnd.randint(1, 4))]
        tail = {n: rnd.random() for lv in levels for _, n in lv}
        allnodes = [x for lv in levels for x in lv]
        want = [n for _, n in sorted(allnodes, key=lambda x: (x[0], tail[x[1]]))[:8]]
        got = _closest_net([list(lv) for lv in levels])
        if got is None:
            seen_tie += 1
            d = sorted(x[0] for x in allnodes)
            assert len(set(d)) < len(d)
        else:
            seen_ok += 1
            assert got == want
    assert seen_tie > 100 and seen_ok > 1000


def _insert_node(lst, x, xbad, SN=14):
    """Search::insertNode (dht.cpp:961-1047, search not expired) on a list of (distance, bad) sorted by distance."""
    if any(d == x for d, _ in lst):
        return
    n = sum(1 for d, _ in lst if d < x)
    bad = sum(b for _, b in lst)
    full = len(lst) - bad >= SN
    t = len(lst)
    while t - bad > SN:
        t -= 1
        if lst[t][1]:
            bad -= 1
    if full:
        del lst[t:]
        if n >= t:
            return
    lst.insert(n, (x, xbad))
    bad += xbad
    while len(lst) - bad > SN:
        bad -= lst[-1][1]
        lst.pop()


def test_search_insert_with_bad_nodes_depends_on_order():
    """Why the swarm's merge with offline peers stays sequential: with bad nodes in play,
    Search::insertNode's list depends on the order of the inserts for some answer sets, so no order-free network can
    stand in for it; without bad nodes it never does (the premise of merge_lookup_net)."""
    rnd = random.Random(5)
    dep = {0.0: 0, 0.2: 0}
    for share in dep:
        for _ in range(3000):
            pool = rnd.sample(range(1000), 60)
            isbad = {x: int(rnd.random() < share) for x in pool}
            base = []
            for x in sorted(rnd.sample(pool, rnd.randint(0, 18))):
                _insert_node(base, x, isbad[x])
            ans = [rnd.choice(pool) for _ in range(rnd.randint(0, 32))]
            res = set()
            for _ in range(6):
                a = list(ans)
                rnd.shuffle(a)
                lst = list(base)
                for x in a:
                    _insert_node(lst, x, isbad[x])
                res.add(tuple(lst))
            dep[share] += len(res) > 1
    assert dep[0.0] == 0 and dep[0.2] > 20
