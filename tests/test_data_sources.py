"""Image sources on the CPU: deterministic synthetic images, JPEG files
(reference naming / Resize+CenterCrop), SDFS shards; ring helpers."""
import io

import numpy as np
import torch

from idunno.runtime.data import JpegSource, SyntheticSource, load_image_u8, synth_images_cpu
from idunno.runtime.executor import TorchExecutor
from idunno.runtime.ring import file_neighbors, neighbors, replica_neighbors


def test_synthetic_deterministic_and_index_addressed():
    a = synth_images_cpu(7, 10, 3)
    b = synth_images_cpu(7, 11, 1)
    assert a.shape == (3, 224, 224, 3) and a.dtype == np.uint8
    assert np.array_equal(a[1], b[0])                     # image i is the same from any chunk
    assert not np.array_equal(a[0], a[1])
    assert abs(a.mean() - 127.5) < 1.0                    # ~uniform bytes
    t = SyntheticSource(7).get(10, 12)
    assert torch.equal(t, torch.from_numpy(a))


def test_jpeg_source_resize_crop(tmp_path):
    from PIL import Image

    rng = np.random.default_rng(0)
    for i, (w, h) in enumerate([(300, 400), (500, 256), (256, 256)]):
        Image.fromarray(rng.integers(0, 256, (h, w, 3), dtype=np.uint8)).save(tmp_path / f"test_{i}.JPEG")
    Image.fromarray(rng.integers(0, 256, (260, 280), dtype=np.uint8), mode="L").save(tmp_path / "test_3.JPEG")
    before = (tmp_path / "test_3.JPEG").read_bytes()
    src = JpegSource("cpu", root=str(tmp_path))
    x = src.get(0, 4)
    assert x.shape == (5, 224, 224, 3) and x.dtype == torch.uint8
    assert src.missing == [4] and x[4].sum() == 0
    assert (tmp_path / "test_3.JPEG").read_bytes() == before   # A14: file not rewritten
    buf = io.BytesIO()
    Image.fromarray(np.full((256, 320, 3), 200, np.uint8)).save(buf, format="PNG")
    y = load_image_u8(buf.getvalue())
    assert y.shape == (224, 224, 3) and int(y[100, 100, 0]) == 200


def test_torch_executor_on_synthetic():
    ex = TorchExecutor("cpu", seed=0)
    imgs = SyntheticSource(3).get(0, 1)
    cls, prob = ex.run("alexnet", imgs, 0, 1)
    assert cls.shape == (2,) and cls.dtype == np.int32 and np.all((prob > 0) & (prob <= 1))
    cls2, _ = ex.run("alexnet", imgs, 0, 1)
    assert np.array_equal(cls, cls2)


def test_ring_helpers_reference_semantics():
    ring = [f"h{i:02d}" for i in range(1, 11)]
    assert replica_neighbors("h05", ring) == ["h06", "h07", "h08", "h09", "h10", "h01", "h02", "h03", "h04", "h05"]
    assert "h03" not in neighbors("h03", ring) and len(neighbors("h03", ring)) == 9
    assert file_neighbors(8, ring, 4) == ["h09", "h10", "h01", "h02"]


def test_deeplearning_api_bs1_cpu_path(tmp_path):
    """Reference L4 API (alexnet_resnet.py:12-92) on the CPU: AlexNet, batch 1
    per forward (BASELINE.json config 1), tuples in the reference format."""
    from PIL import Image

    from idunno.inference import deeplearning

    res, dt = deeplearning("nope", "alexnet", 5, 7, device="cpu", batch=1, root=str(tmp_path))
    assert [r[0] for r in res] == ["test_5.JPEG", "test_6.JPEG", "test_7.JPEG"] and dt > 0
    assert all(isinstance(c, str) and 0 < p <= 1 for _, c, p in res)
    # batched forward gives the same answers as batch 1
    res_b, _ = deeplearning("nope", "alexnet", 5, 7, device="cpu", root=str(tmp_path))
    assert [r[1] for r in res_b] == [r[1] for r in res]
    assert max(abs(a[2] - b[2]) for a, b in zip(res, res_b)) < 1e-4
    # a ./<filename>/test_<i>.JPEG directory is used when it exists
    d = tmp_path / "resnet"
    d.mkdir()
    Image.fromarray(np.full((256, 256, 3), 90, np.uint8)).save(d / "test_0.JPEG")
    res_j, _ = deeplearning("resnet", "resnet", 0, 0, device="cpu", root=str(tmp_path))
    assert len(res_j) == 1 and res_j[0][0] == "test_0.JPEG"


class _ShardStore:
    """Minimal SDFS stand-in: shard bytes by name, with a read counter."""

    def __init__(self, seed, n, per):
        from idunno.runtime.data import shard_name

        self.files = {shard_name(k): synth_images_cpu(seed, k * per, min(per, n - k * per)).tobytes()
                      for k in range(-(-n // per))}
        self.reads = []

    def get_bytes_ver(self, name):
        self.reads.append(name)
        d = self.files.get(name)
        return None if d is None else (d, 1)

    def fetch_hbm(self, name, device):
        return None

    def announce_hbm(self, *a, **k):
        pass


def test_sdfs_source_readahead_prefetches_next_shard():
    """A request for shard k starts shard k+1 in the background (sequential
    readahead), so the next chunk's read + H2D overlap the current compute."""
    import time

    from idunno.runtime.data import SdfsSource, shard_name

    store = _ShardStore(5, 30, 10)
    src = SdfsSource(store, "cpu", shard_images=10, peer_copy=False, readahead=1)
    x = src.get(0, 9)
    assert torch.equal(x, torch.from_numpy(synth_images_cpu(5, 0, 10)))
    for _ in range(200):                                 # shard 1 lands in the background
        if src.cached(10, 19):
            break
        time.sleep(0.01)
    assert src.cached(10, 19) and store.reads[:2] == [shard_name(0), shard_name(1)]
    y = src.get(12, 21)                                  # spans shards 1 and 2: 1 cached, 2 prefetched by now or fetched
    assert torch.equal(y, torch.from_numpy(synth_images_cpu(5, 12, 10)))
    assert store.reads.count(shard_name(1)) == 1        # never read twice
    src.get(25, 29)                                      # readahead past the last shard: harmless
    assert torch.equal(src.get(20, 29), torch.from_numpy(synth_images_cpu(5, 20, 10)))


def test_stage_file_parallel_preadv(tmp_path):
    """HbmStager.stage_file reads a file with parallel preadv calls straight
    into its buffers (CPU here; pinned ping-pong + side-stream DMA on a GPU)."""
    from idunno.runtime.data import HbmStager

    data = np.random.default_rng(1).integers(0, 256, 20 << 20, dtype=np.uint8)
    p = tmp_path / "blob"
    p.write_bytes(data.tobytes() + b"tail")               # longer than the staged shape: ignored
    st = HbmStager("cpu")
    t = st.stage_file(str(p), (20, 1 << 20))
    assert t.shape == (20, 1 << 20) and np.array_equal(t.reshape(-1).numpy(), data)
    try:
        st.stage_file(str(p), (21, 1 << 20))
        raise AssertionError("short file accepted")
    except ValueError:
        pass


def test_sdfs_source_streams_local_replica_file(tmp_path):
    """A shard this node holds a replica of is streamed from its file
    (``local_file``) instead of coming back as a bytes object."""
    from idunno.runtime.data import SdfsSource, shard_name

    class LocalStore(_ShardStore):
        def local_file(self, name):
            d = self.files.get(name)
            if d is None or name == shard_name(2):         # shard 2: another node's replica
                return None
            p = tmp_path / name.replace("/", "_")
            p.write_bytes(d)
            return str(p), 1

    store = LocalStore(6, 30, 10)
    src = SdfsSource(store, "cpu", shard_images=10, peer_copy=False, readahead=0)
    x = src.get(0, 29)
    assert torch.equal(x, torch.from_numpy(synth_images_cpu(6, 0, 30)))
    assert src.local_reads == 2 and store.reads == [shard_name(2)]


def test_sdfs_source_prefetch_range_stages_in_background():
    """SdfsSource.prefetch(start, end): every shard of the range is staged by
    the readahead thread before any get() asks for it."""
    import time

    from idunno.runtime.data import SdfsSource, shard_name

    store = _ShardStore(8, 40, 10)
    src = SdfsSource(store, "cpu", shard_images=10, peer_copy=False, readahead=0)
    src.prefetch(5, 34)                                  # shards 0..3
    for _ in range(300):
        if src.cached(0, 39):
            break
        time.sleep(0.01)
    assert src.cached(0, 39) and sorted(store.reads) == [shard_name(k) for k in range(4)]
    assert torch.equal(src.get(5, 34), torch.from_numpy(synth_images_cpu(8, 5, 30)))
    assert len(store.reads) == 4                         # nothing read twice


def test_resident_source_cpu_falls_back_to_synthetic():
    """On a CPU device ResidentSource keeps nothing resident and serves every
    request as SyntheticSource would (same bytes); is_resident() is false for
    ordinary tensors (so the executor never takes the window path for them)."""
    from idunno.runtime.data import ResidentSource, SyntheticSource, is_resident

    src = ResidentSource(5, "cpu")
    src.make_resident(100)
    assert src.data is None
    a = src.get(10, 19)
    assert torch.equal(a, SyntheticSource(5, "cpu").get(10, 19))
    assert not is_resident(a) and not is_resident(torch.zeros(3))
