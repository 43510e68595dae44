"""Model families of the reference (AlexNet, ResNet18) plus ResNet34/50.

``reference``  plain-PyTorch fp32 oracle modules (torchvision-compatible keys)
``packed``     BN-folded, MFMA-packed inference programs + HIP runner
"""
from . import reference
from .packed import HipRunner, Program, build_program, compile_model, emulate, program_flops
from .reference import canonical

__all__ = ["reference", "HipRunner", "Program", "build_program", "compile_model", "emulate",
           "program_flops", "canonical"]
