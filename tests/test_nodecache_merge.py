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
