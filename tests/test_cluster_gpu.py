"""Cluster path on the GPU: HIP executor + synthetic / SDFS-staged image
sources, several nodes sharing cuda:0 (one MI355X box)."""
import ast

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

FAST = dict(heartbeat_period_s=0.05, failure_timeout_s=1.0, metadata_period_s=0.2, rpc_timeout_s=10.0)


def test_synthetic_images_cpu_gpu_identical():
    from idunno import ops
    from idunno.runtime.data import synth_images_cpu

    a = synth_images_cpu(1234, 37, 5)
    b = ops.synth_images(1234, 37, 5, "cuda").cpu().numpy()
    assert a.shape == (5, 224, 224, 3) and np.array_equal(a, b)


def test_hbm_stager_roundtrip():
    from idunno.runtime.data import HbmStager

    st = HbmStager(torch.device("cuda"), pinned_bytes=1 << 20)
    data = np.random.default_rng(0).integers(0, 256, size=3 * 224 * 224 * 3 + 0, dtype=np.uint8)
    t = st.stage(data.tobytes(), (3, 224, 224, 3))
    assert t.is_cuda and np.array_equal(t.cpu().numpy().reshape(-1), data)


@pytest.mark.parametrize("pinned_mb,threads", [(1, 8), (64, 8), (3, 1)])
def test_hbm_stager_file_native(tmp_path, pinned_mb, threads):
    """HbmStager.stage_file through the extension's GIL-free stager
    (csrc/runtime/staging.cpp): byte-exact against the file for sizes that are
    not a multiple of the pinned pieces, then the pinned buffers are reusable by
    the Python byte path; the Python preadv path gives the same bytes."""
    from idunno import ops
    from idunno.runtime.data import HbmStager

    assert hasattr(ops.load(), "stage_file_native")
    rng = np.random.default_rng(pinned_mb + threads)
    data = rng.integers(0, 256, size=(9 << 20) + 4099, dtype=np.uint8)
    p = tmp_path / "shard.bin"
    p.write_bytes(data.tobytes())
    st = HbmStager(torch.device("cuda"), pinned_bytes=pinned_mb << 20)
    st.READ_THREADS = threads
    assert st._native() is not None
    t = st.stage_file(str(p), (data.size,))
    assert t.is_cuda and np.array_equal(t.cpu().numpy(), data)
    t2 = st.stage(data[:1000].tobytes(), (1000,))
    assert np.array_equal(t2.cpu().numpy(), data[:1000])
    with pytest.raises(Exception):
        st.stage_file(str(tmp_path / "missing.bin"), (10,))
    import os

    os.environ["IDUNNO_PY_STAGING"] = "1"
    try:
        assert st._native() is None
        t3 = st.stage_file(str(p), (data.size,))
        assert np.array_equal(t3.cpu().numpy(), data)
    finally:
        os.environ.pop("IDUNNO_PY_STAGING")


def _cluster(source_kind):
    from idunno.runtime.cluster import LocalCluster
    from idunno.runtime.data import SdfsSource, SyntheticSource
    from idunno.runtime.executor import HipExecutor

    def src(i, node):
        if source_kind == "sdfs":
            return SdfsSource(node.sdfs, "cuda", shard_images=50)
        return SyntheticSource(node.cfg.data_seed, "cuda")

    return LocalCluster(num_nodes=3, executor_factory=lambda i: HipExecutor("cuda", seed=0),
                        source_factory=src, **FAST).start()


def _collect(cl, model, n):
    res = cl.view("c4")["results"]
    got = {}
    for k, chunks in res.items():
        if k.startswith(model + " "):
            for ch in chunks:
                for name, cat, p in ast.literal_eval(ch):
                    got[int(name[5:-5])] = (int(cat.split("_")[1]), p)
    assert sorted(got) == list(range(n))
    return got


def test_cluster_hip_vs_fp32_oracle_and_sdfs_path():
    from idunno.models import reference as ref
    from idunno.runtime.data import put_synthetic_dataset, synth_images_cpu

    c = _cluster("synthetic")
    try:
        cl = c.client()
        cl.inference(0, 199, "resnet18")
        assert cl.wait_idle(120, {"resnet18": 200})["done"]["resnet18"] == 200
        got = _collect(cl, "resnet18", 200)
    finally:
        c.stop()
    from idunno.models import HipRunner, build_program

    imgs = torch.from_numpy(synth_images_cpu(c.cfg.data_seed, 0, 200)).cuda()
    # the cluster path (split, dispatch, graphs per chunk size, gather) must give
    # exactly what one direct forward of the same kernels gives
    dc, dp = HipRunner(build_program("resnet18", seed=0)).forward(imgs)
    assert all(got[i][0] == dc[i].item() for i in range(200))
    # and the probabilities must match the fp32 oracle's probability of that class
    # (default-init ResNet18 on noise has near-tied logits, so argmax equality
    # with the oracle is not a meaningful check here; kernel tests cover it)
    m = ref.build("resnet18", seed=0).cuda()
    with torch.no_grad():
        p = torch.softmax(m(ref.preprocess_u8(imgs)), 1)
    perr = max(abs(got[i][1] - p[i, got[i][0]].item()) for i in range(200))
    assert perr < 0.02 * p.max().item() + 1e-4, perr

    c2 = _cluster("sdfs")
    try:
        put_synthetic_dataset(c2.nodes["node00"].sdfs, 200, c2.cfg.data_seed, shard_images=50)
        cl2 = c2.client()
        cl2.inference(0, 199, "resnet18")
        assert cl2.wait_idle(120, {"resnet18": 200})["done"]["resnet18"] == 200
        got2 = _collect(cl2, "resnet18", 200)
    finally:
        c2.stop()
    # same images, same kernels: bit-identical answers whichever path fed them
    assert all(got2[i][0] == got[i][0] for i in range(200))


def test_sdfs_shard_peer_copy_between_nodes():
    """A shard one node holds in HBM reaches another node as a GPU-to-GPU copy
    (SDFS FETCH_HBM), not through a replica read + host staging."""
    from idunno.runtime.data import put_synthetic_dataset, synth_images_cpu

    c = _cluster("sdfs")
    try:
        put_synthetic_dataset(c.nodes["node00"].sdfs, 100, c.cfg.data_seed, shard_images=50)
        a, b = c.nodes["node01"], c.nodes["node02"]
        # no readahead: node01 must hold shard 0 only (its background fetch of
        # shard 1 would make that a peer copy too, depending on timing)
        a.source.readahead = b.source.readahead = 0
        ta = a.source.get(0, 49)
        torch.cuda.synchronize()
        assert a.source.peer_fetches == 0
        tb = b.source.get(10, 59)                 # shard 0 from node01's HBM, shard 1 from a replica
        torch.cuda.synchronize()
        assert b.source.peer_fetches == 1 and b.sdfs.peer_copies == 1
        want = torch.from_numpy(synth_images_cpu(c.cfg.data_seed, 0, 60)).cuda()
        assert torch.equal(ta, want[:50]) and torch.equal(tb, want[10:60])
    finally:
        c.stop()


def _eager(ex, model, imgs):
    r = ex.runner(model)
    cls, prob = r.forward(imgs.contiguous())
    torch.cuda.synchronize()
    return cls.cpu().numpy(), prob.cpu().numpy()


def test_hip_executor_two_threads_same_batch():
    """chunks of two threads (TCP worker + round driver) through one
    executor, same chunk size, different images: results never mix."""
    import threading

    from idunno import ops
    from idunno.runtime.executor import HipExecutor

    ex = HipExecutor("cuda", seed=0)
    imgs = [ops.synth_images(100 + i, 0, 48, "cuda") for i in range(6)]
    want = [_eager(ex, "resnet18", im) for im in imgs]
    got = {}
    errs = []

    def worker(ids):
        try:
            for _ in range(3):
                for i in ids:
                    got.setdefault(i, []).append(ex.run("resnet18", imgs[i], 0, 47))
        except Exception as e:  # noqa: BLE001
            errs.append(e)

    ts = [threading.Thread(target=worker, args=(ids,)) for ids in ((0, 1, 2), (3, 4, 5))]
    for t in ts:
        t.start()
    for t in ts:
        t.join(120)
    assert not errs, errs
    for i in range(6):
        for cls, prob in got[i]:
            assert np.array_equal(cls, want[i][0]) and np.allclose(prob, want[i][1], rtol=0, atol=0)
    ex.close()


def test_hip_executor_submit_two_in_flight():
    """submit() launches up to two chunks before their read-back; a third
    waits for a free slot; every result matches the eager forward."""
    import threading

    from idunno import ops
    from idunno.runtime.executor import HipExecutor

    ex = HipExecutor("cuda", seed=0)
    imgs = [ops.synth_images(200 + i, 0, 40, "cuda") for i in range(3)]
    want = [_eager(ex, "resnet18", im) for im in imgs]
    a = ex.submit("resnet18", imgs[0], 0, 39)
    b = ex.submit("resnet18", imgs[1], 0, 39)
    third = {}
    t = threading.Thread(target=lambda: third.setdefault("h", ex.submit("resnet18", imgs[2], 0, 39)))
    t.start()
    t.join(0.5)
    assert t.is_alive()                    # both slots busy
    ra = a.result()
    t.join(60)
    assert not t.is_alive()
    rb, rc = b.result(), third["h"].result()
    for (cls, prob), (wc, wp) in zip((ra, rb, rc), want):
        assert np.array_equal(cls, wc) and np.array_equal(prob, wp)
    ex.close()


def test_run_packed_resident_window_matches_copy():
    """run_packed on views of a ResidentSource reads the images in place (window
    graph, device-side start) and gives the same (class, prob) as a copy of the
    same images; a view at a new offset reuses the graph (no new capture)."""
    from idunno.runtime.data import ResidentSource, synth_images_cpu
    from idunno.runtime.executor import HipExecutor

    ex = HipExecutor("cuda", seed=0)
    src = ResidentSource(7, "cuda")
    src.make_resident(200)
    assert torch.equal(src.get(30, 35).cpu(), torch.from_numpy(synth_images_cpu(7, 30, 6)))
    packed = torch.zeros(64, 2, dtype=torch.int32, device="cuda")
    r = ex.runner("resnet18")
    for start in (0, 40, 136):
        view = src.get(start, start + 47)
        assert view._base is not None
        ex.run_packed("resnet18", view, packed[:48])
        torch.cuda.synchronize()
        got = packed[:48].clone()
        ngraphs = len(r._graphs)
        want_cls, want_prob = _eager(ex, "resnet18", view.clone())
        assert np.array_equal(got[:, 0].cpu().numpy(), want_cls)
        assert np.array_equal(got[:, 1].cpu().numpy().view(np.float32), want_prob)
        assert r.has_window(src.data, 48, packed=packed[:48])
    assert len(r._graphs) == ngraphs
    assert src.get(195, 205).shape[0] == 11         # past the resident range: generated per request
    # a view of any other tensor (an SDFS shard) keeps the static-input graph
    other = src.data.clone()
    n0 = len(r._graphs)
    ex.run_packed("resnet18", other[8:56], packed[:48])
    torch.cuda.synchronize()
    assert not r.has_window(other, 48, packed=packed[:48]) and len(r._graphs) <= n0 + 1
    ex.close()
