"""HipExecutor on the GPU: chunks of several sizes, interleaved and two in
flight, through graphs that share ONE memory pool (round 6: a pool per graph
ran 8 node processes sharing one GPU out of memory once the fair-time split
re-planned chunk sizes).  Every chunk must equal an eager forward of the same
images, and the shared pool must hold less than separate pools would."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_shared_pool_graphs_interleaved_sizes():
    from idunno import ops
    from idunno.runtime.executor import HipExecutor

    dev = torch.device("cuda:0")
    ex = HipExecutor(dev, seed=3, dtype="fp16")
    imgs = ops.synth_images(11, 0, 96, dev)
    r = ex.runner("resnet18")
    assert r.graph_pool is not None
    sizes = [8, 24, 8, 40, 24, 16, 40, 8]
    pend, starts, got = [], [], []
    s0 = 0
    for n in sizes:
        if len(pend) == 2:                           # the executor has two launch slots
            got.append(pend.pop(0).result())
        starts.append(s0)
        pend.append(ex.submit("resnet18", imgs[s0:s0 + n], s0, s0 + n - 1))
        s0 = (s0 + 7) % 50
    got += [p.result() for p in pend]
    for (cls, prob), n, s in zip(got, sizes, starts):
        want_c, want_p = r.forward(imgs[s:s + n].contiguous())
        torch.cuda.synchronize()
        assert np.array_equal(cls, want_c.cpu().numpy().astype(np.int32)), (n, s)
        assert np.allclose(prob, want_p.float().cpu().numpy(), rtol=0, atol=1e-6), (n, s)
    assert len(r._graphs) >= 4                       # one graph per size and slot
    ex.close()


def test_failed_capture_falls_back_to_eager():
    """A capture that fails (out of memory in a crowded GPU) must not fail the
    chunk: the executor runs it eagerly and captures nothing more."""
    from idunno import ops
    from idunno.runtime.executor import HipExecutor

    dev = torch.device("cuda:0")
    ex = HipExecutor(dev, seed=4, dtype="fp16")
    imgs = ops.synth_images(12, 0, 16, dev)
    r = ex.runner("resnet18")
    pool0 = r.graph_pool

    def boom(*a, **k):
        raise torch.cuda.OutOfMemoryError("synthetic capture failure")

    r.capture = boom
    cls, prob = ex.run("resnet18", imgs, 0, 15)
    want_c, want_p = r.forward(imgs)
    torch.cuda.synchronize()
    assert np.array_equal(cls, want_c.cpu().numpy().astype(np.int32))
    assert ex.graphs_broken and r.graph_pool is not pool0 and not r._graphs
    cls2, _ = ex.run("resnet18", imgs, 0, 15)          # eager from now on
    assert np.array_equal(cls2, cls)
    ex.close()
