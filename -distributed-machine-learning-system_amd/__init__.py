"""IDunno-MI355X: a fault-tolerant distributed image-classification inference
cluster for one AMD MI355X node (8 x gfx950), re-designed from the CS425
"IDunno" reference (kentchen831213/-Distributed-Machine-Learning-System).

Layers:
  config        typed configuration (L0)
  runtime/      transport, membership + failure detector, SDFS, scheduler,
                coordinator / hot standby, job-state tables, shell (L1-L7)
  parallel/     one-process-per-GPU RCCL data plane (dispatch, top-1 gather)
  models/       AlexNet / ResNet programs and the HIP runner (L4)
  ops/          gfx950 HIP kernels (implicit-GEMM MFMA conv, pools, softmax-top1)
"""
__version__ = "0.1.0"
