"""HSR_Net multimodal fusion producer -- the module that turns the raw sensor
streams into the [N x 1728] windows the autoencoder consumes.

Mirrors ``utils/data_loaders.py:152-229`` (``HSR_Net(unimodal, config)``,
``forward(r, d, l, t, m)``): the same conv submodules (so ``state_dict`` keys
and shapes match the reference, including the unused LiDAR / ``conv1m`` /
``conv2m`` ones), torch's default init, and the same output shapes
([n, 27, 8, 8] fused; [n, 16|8|1|2, 8, 8] unimodal).  The reference loops over
``config.slicing_size`` windows in Python and concatenates per window
(:183-228); here the whole batch is ONE native call (``mmad_hsr_fuse``,
``include/mmad.h``; kernel ``csrc/mmad_hsr.hip``).  No CPU fallback: without
the library or a GPU the forward raises ``NativeUnavailable``.
"""
import torch
from torch import nn

from . import _native

# modality -> (channels of its 8x8 block, packed row width)
_BLOCK = {"r": 16, "d": 8, "t": 1, "m": 2}
# parameters the kernel reads, in the packed order of mmad_hsr_fuse
_PACKED = ("conv1r", "conv2r", "conv3r", "conv1d", "conv2d", "conv3d", "conv1l", "conv2l")


class HSR_Net(nn.Module):
    """utils/data_loaders.py:151-229."""

    def __init__(self, unimodal, config):
        super().__init__()
        self.conv1r = nn.Conv2d(3, 16, kernel_size=2, stride=2)
        self.conv2r = nn.Conv2d(16, 16, kernel_size=3, stride=1, padding=1)
        self.conv3r = nn.Conv2d(16, 16, kernel_size=2, stride=2)

        self.conv1d = nn.Conv2d(1, 8, kernel_size=2, stride=2)
        self.conv2d = nn.Conv2d(8, 8, kernel_size=3, stride=1, padding=1)
        self.conv3d = nn.Conv2d(8, 8, kernel_size=2, stride=2)
        self.batch_size = config.slicing_size
        self.config = config

        self.conv1l = nn.Conv1d(1, 8, kernel_size=18, stride=9, padding=9)
        self.conv2l = nn.Conv1d(8, 16, kernel_size=2, stride=2)
        self.conv3l = nn.Conv1d(16, 32, kernel_size=2, stride=2)
        self.conv4l = nn.Conv1d(32, 16, kernel_size=3, stride=2, padding=3)
        self.conv5l = nn.Conv1d(16, 32, kernel_size=2, stride=2)

        self.conv1m = nn.Conv1d(1, 12, kernel_size=2, stride=1)
        self.conv2m = nn.Conv1d(12, 8, kernel_size=2, stride=2, padding=2)
        self.unimodal = unimodal

    def packed_weights(self):
        """fp32 [mmad_hsr_weight_count()] on the module's device (conv1r w, b, ...)."""
        parts = []
        for name in _PACKED:
            conv = getattr(self, name)
            parts += [conv.weight.detach().reshape(-1), conv.bias.detach().reshape(-1)]
        w = torch.cat(parts).float().contiguous()
        n = _native.load().mmad_hsr_weight_count()
        if w.numel() != n:
            raise _native.NativeError(f"hsr weights: packed {w.numel()} floats, kernel expects {n}")
        return w

    def forward(self, r, d, l, t, m, out=None):
        """Fuse ``config.slicing_size`` windows (data_loaders.py:183-229).
        ``out`` (optional): a preallocated fp32 [n, >= width] device tensor to
        fill (e.g. wider rows padded for the autoencoder); returned as a view."""
        if l is not None:
            raise NotImplementedError("HSR_Net LiDAR branch: the reference never feeds it "
                                      "(utils/data_loaders.py:401, :405-424)")
        given = {k: v for k, v in (("r", r), ("d", d), ("t", t), ("m", m)) if v is not None}
        if not self.unimodal and len(given) < 4:
            missing = [k for k in "rdtm" if k not in given]
            # the reference's torch.cat((rr, dd, tt, mm)) hits an unbound name
            raise NameError(f"HSR_Net: fused output needs r, d, t and m; missing {missing}")
        if self.unimodal and not given:
            raise UnboundLocalError("HSR_Net: unimodal forward with no modality (no result)")
        n = int(self.batch_size)
        for k, v in given.items():
            if v.shape[0] < n:
                raise IndexError(f"HSR_Net: {k} has {v.shape[0]} windows < slicing_size {n}")
        w = self.packed_weights()
        _native.require_gpu(w)
        per = {"r": 3 * 32 * 32, "d": 32 * 32, "t": 1, "m": 13}
        flat = {}
        for k, v in given.items():
            x = v[:n].reshape(n, -1)
            if x.shape[1] != per[k]:
                raise ValueError(f"HSR_Net: {k} windows have {x.shape[1]} values, expected {per[k]}")
            flat[k] = x.to(device=w.device, dtype=torch.float32).contiguous()
        keep = list(given)[-1] if self.unimodal else None
        chans = _BLOCK[keep] if keep else sum(_BLOCK.values())
        width = chans * 64
        if out is None:
            out = torch.empty(n, width, device=w.device, dtype=torch.float32)
        if (not out.is_cuda or out.dtype != torch.float32 or out.dim() != 2 or out.shape[0] < n
                or out.shape[1] < width or out.stride(1) != 1):
            raise ValueError("HSR_Net: out must be a row-major fp32 device tensor [n, >= width]")
        ptr = _native.ptr
        sel = (lambda k: flat[k] if (k in flat and (keep is None or k == keep)) else None)
        _native.call("mmad_hsr_fuse", n, ptr(sel("r")), ptr(sel("d")), ptr(sel("t")), ptr(sel("m")),
                     ptr(w), 1 if self.unimodal else 0, ptr(out), out.stride(0),
                     _native.stream_ptr())
        return out[:n, :width].view(n, chans, 8, 8) if out.stride(0) == width else out[:n, :width]
