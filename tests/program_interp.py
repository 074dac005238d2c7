"""Test-only CPU interpreter of a planned codec program (gpi/plan.py).

Executes the op list with torch ops, reading each op's channel ranges,
BN parameter names and conv geometry exactly as the HIP kernels do, so the
planner's wiring (buffers, channel offsets, concat-in-place, BN placement)
is validated on CPU against the oracle codec.  Never used by the product.
"""
import torch
import torch.nn.functional as F


def run_program(prog, params, x, groups=None):
    """prog: CodecProgram; params: name -> tensor; x: input [B, C, H, W]."""
    B = x.shape[0]
    groups = groups or [B]
    bufs = {}
    for b in prog.buffers:
        bufs[id(b)] = torch.zeros(B, b.C, b.H, b.W, dtype=x.dtype)
    bufs[id(prog.input)] = x
    for op in prog.ops:
        src = bufs[id(op.src)][:, op.c0:op.c0 + op.cin]
        if op.bn is not None:
            outs = []
            s = 0
            for n in groups:
                outs.append(F.batch_norm(src[s:s + n], None, None, params[op.bn + '.weight'],
                                         params[op.bn + '.bias'], training=True, eps=1e-5))
                s += n
            src = torch.relu(torch.cat(outs, 0))
        if op.upsample:
            src = F.interpolate(src, scale_factor=2.0, mode='nearest')
        y = F.conv2d(src, params[op.w], stride=op.stride, padding=op.pad)
        dst = bufs[id(op.dst)].clone()
        dst[:, op.d0:op.d0 + op.cout] = y
        bufs[id(op.dst)] = dst
    return bufs[id(prog.output)]
