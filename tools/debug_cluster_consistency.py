#!/usr/bin/env python3
"""Diagnose cluster-path vs direct-forward differences on the GPU."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from idunno.models import HipRunner, build_program
    from idunno.runtime.data import SyntheticSource, synth_images_cpu
    from idunno.runtime.executor import HipExecutor

    seed = 1234
    imgs = torch.from_numpy(synth_images_cpu(seed, 0, 200)).cuda()
    src = SyntheticSource(seed, "cuda")
    g = src.get(0, 199)
    print("synth cpu==gpu:", torch.equal(imgs, g))
    r = HipRunner(build_program("resnet18", seed=0))
    l_all = r.logits(imgs)
    c_all, p_all = r.forward(imgs)
    for n in (67, 66, 1, 16):
        l_n = r.logits(imgs[:n].contiguous())
        print(f"eager n={n}: max|dlogit|={(l_n - l_all[:n]).abs().max().item():.3e}")
    ex = HipExecutor("cuda", seed=0)
    for (s, e) in ((0, 66), (67, 133), (134, 199)):
        cls, prob = ex.run("resnet18", src.get(s, e), s, e)
        ref_c = c_all[s:e + 1].cpu().numpy()
        ref_p = p_all[s:e + 1].cpu().numpy()
        print(f"executor chunk [{s},{e}] cls mismatches={int((cls != ref_c).sum())} max|dp|={abs(prob - ref_p).max():.3e}")
    sin, run = r.capture(67)
    sin.copy_(imgs[:67])
    c_g, p_g = run()
    torch.cuda.synchronize()
    print("graph n=67 mismatches:", int((c_g != c_all[:67]).sum().item()), "max|dp|", (p_g - p_all[:67]).abs().max().item())
    # concurrency: 3 executors in 3 threads on one GPU, like 3 nodes of a LocalCluster
    import threading

    for use_graphs in (False, True):
        exs = [HipExecutor("cuda", seed=0, use_graphs=use_graphs) for _ in range(3)]
        chunks = [(0, 66), (67, 133), (134, 199)]
        res = {}

        def work(k):
            s, e = chunks[k]
            for rep in range(3):
                imgs_k = src.get(s, e)
                res[(k, rep)] = exs[k].run("resnet18", imgs_k, s, e)

        ths = [threading.Thread(target=work, args=(k,)) for k in range(3)]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        bad = 0
        for (k, rep), (cls, prob) in sorted(res.items()):
            s, e = chunks[k]
            mism = int((cls != c_all[s:e + 1].cpu().numpy()).sum())
            bad += mism
            print(f"threads graphs={use_graphs} chunk {k} rep {rep}: mismatches={mism}")
        print(f"threads graphs={use_graphs}: total mismatches {bad}")
    top2 = torch.topk(l_all, 2, dim=1).values
    print("median top1-top2 logit margin:", (top2[:, 0] - top2[:, 1]).median().item(),
          "logit scale:", l_all.abs().max().item())


if __name__ == "__main__":
    main()
