"""Line sets built on first use (kadgpu.h KAD_TABLE_EAGER / kad_table_prepare): a table is created with the
count <= 8 lines only; the count 9..32 RoutingTable lines and the NodeCache lines are built by the first query
that needs them (never inside a graph capture, where the query answers on its exact path), and are then kept
current by status refreshes like the others. Results are identical to an eagerly built table and to the
oracle."""
import numpy as np
import pytest
import torch

import oracle as O
import tables as TB
from opendht_amd import DeviceTable

pytestmark = pytest.mark.gpu


def _dev(a, gpu):
    return torch.from_numpy(np.ascontiguousarray(a)).to(gpu)


def test_bench_shard_k8_footprint(gpu):
    """The bench shard (1/8 of the 100M-node table) answering k = 8 holds < 1 GB of HBM (round 2: 4.8 GB, every
    line set eager); the other sets appear with their first query."""
    from opendht_amd.sharded import build_shard, config3_spec

    sh = build_shard(config3_spec(), 0)
    tg = _dev(config3_spec().targets_for(0, 1 << 16, seed=9), gpu)
    with DeviceTable(sh.ids, sh.status, sh.first, sh.off, device=0, index_base=sh.index_base, sorted=True) as T:
        T.rt_closest(tg, 8)
        torch.cuda.synchronize()
        inf = T.info()
        print({k: v for k, v in inf.items() if k in ("device_bytes", "line_sets")})
        assert inf["device_bytes"] < 1 << 30
        assert not any(v["built"] for v in inf["line_sets"].values())
        T.rt_closest(tg, 14)
        T.nc_closest(tg, 14)
        torch.cuda.synchronize()
        ls = T.info()["line_sets"]
        assert ls["rt16"]["built"] and ls["rt32"]["built"] and ls["nc16"]["built"] and not ls["nc32"]["built"]
        assert ls["rt16"]["bytes"] > 0 and ls["nc16"]["build_ms"] > 0


@pytest.mark.parametrize("t", [TB.uniform_config(120_000, 14, seed=0x15E), TB.split_config(60_000, seed=0x15F)],
                         ids=lambda t: t["name"])
def test_lazy_equals_eager_and_follows_refresh(gpu, t):
    targets = TB.adversarial_targets(t, extra=3000)
    tg = _dev(targets, gpu)
    rng = np.random.default_rng(3)
    srt = t["sorted"]
    with DeviceTable(t["ids"], t["status"], t["first"], t["off"], device=0, sorted=srt) as L, \
            DeviceTable(t["ids"], t["status"], t["first"], t["off"], device=0, sorted=srt, eager=True) as E:
        assert E.info()["line_sets"]["rt32"]["built"]
        assert E.info()["line_sets"]["nc16"]["built"] == srt and E.info()["line_sets"]["nc32"]["built"] == srt
        st = t["status"]
        for rep in range(2):
            for k in (8, 14, 16, 24, 32):
                a, ac = L.rt_closest(tg, k)
                b, bc = E.rt_closest(tg, k)
                torch.cuda.synchronize()
                want, wcnt = O.flat_rt_closest(t["ids"], st, t["first"], t["off"], targets, k, nthreads=8)
                np.testing.assert_array_equal(a.cpu().numpy().view(np.uint32), want, err_msg=f"lazy k={k} rep={rep}")
                np.testing.assert_array_equal(b.cpu().numpy().view(np.uint32), want, err_msg=f"eager k={k} rep={rep}")
                np.testing.assert_array_equal(ac.cpu().numpy(), wcnt)
            for k in ((14, 32) if srt else ()):
                a, ac = L.nc_closest(tg, k)
                torch.cuda.synchronize()
                want, wcnt = O.flat_nc_closest(t["ids"], st, targets, k, nthreads=8)
                np.testing.assert_array_equal(a.cpu().numpy().view(np.uint32), want, err_msg=f"lazy nc k={k}")
            # a status change after the sets were built: they are rebuilt incrementally with the others
            nodes = rng.choice(t["ids"].shape[0], size=t["ids"].shape[0] // 50, replace=False).astype(np.uint32)
            st = st.copy()
            st[nodes] = rng.choice(np.array([0, 1, 2], np.uint8), size=nodes.shape[0])
            L.patch_status(nodes, st[nodes])
            E.patch_status(nodes, st[nodes])


def test_graph_capture_before_and_after_prepare(gpu):
    """A query captured in a HIP graph on a table whose set is not built answers on its exact path (no allocation
    inside the capture); after prepare() the captured query uses the lines. Both replay bit-exact."""
    t = TB.uniform_config(100_000, 14, seed=0x160)
    targets = TB.adversarial_targets(t, extra=2000)
    tg = _dev(targets, gpu)
    want, wcnt = O.flat_rt_closest(t["ids"], t["status"], t["first"], t["off"], targets, 14, nthreads=8)
    with DeviceTable(t["ids"], t["status"], t["first"], t["off"], device=0, sorted=True) as T:
        for prepared in (False, True):
            if prepared:
                T.prepare()
            out = torch.empty((targets.shape[0], 14), dtype=torch.int32, device=gpu)
            cnt = torch.empty((targets.shape[0],), dtype=torch.uint8, device=gpu)
            g = torch.cuda.CUDAGraph()
            s = torch.cuda.Stream(gpu)
            s.wait_stream(torch.cuda.current_stream(gpu))
            with torch.cuda.graph(g, stream=s):
                T.rt_closest(tg, 14, out, cnt, stream=s.cuda_stream)
            assert T.info()["line_sets"]["rt16"]["built"] == prepared
            out.fill_(-7)
            g.replay()
            torch.cuda.synchronize()
            np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), want, err_msg=f"prepared={prepared}")
            np.testing.assert_array_equal(cnt.cpu().numpy(), wcnt)
