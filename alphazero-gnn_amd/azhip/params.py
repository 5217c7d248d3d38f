"""Flat parameter storage: one contiguous fp32 HBM buffer per network (+ grad / Adam moments),
with a named view per tensor in the reference's state_dict order.  One buffer means one Adam
launch and one all-reduce bucket per network; every tensor starts on a 16-byte boundary so
the kernels can read it with 16-byte loads."""
from collections import OrderedDict

import numpy as np
import torch


def weights_changed():
    """Tell libaz_hip.so that parameter values changed (az_weights_changed): the fp16 GEMM form
    recomputes its cached per-row weight scales before their next use.  Every in-place write of
    a parameter buffer outside az_adam_f32 must call this (load_state_dict, copy_flat_ do)."""
    if not torch.cuda.is_available():
        return
    from . import _lib
    _lib.check(_lib.load().az_weights_changed(), "az_weights_changed")


def _register(owner, flat):
    """Declare `flat` parameter storage to libaz_hip.so (az_weights_register: its weights' fp16
    GEMM scales / planes may be cached between az_weights_changed calls) for as long as `owner`
    lives."""
    if flat.device.type != "cuda" or flat.numel() == 0:
        return
    import weakref
    from . import _lib
    L = _lib.load()
    ptr = flat.data_ptr()
    _lib.check(L.az_weights_register(ptr, flat.numel() * 4), "az_weights_register")
    # the buffer outlives the owner only through views; unregistering early only disables caching.
    # Not at interpreter exit: the library frees its cache entries then, and the HIP runtime may
    # already be going down.
    weakref.finalize(owner, L.az_weights_unregister, ptr).atexit = False


def _align4(n):
    return (n + 3) & ~3


class FlatParams:
    def __init__(self, spec, device, init=None):
        self.spec = list(spec)
        self.device = torch.device(device)
        self.offsets = OrderedDict()
        off = 0
        for name, shape in self.spec:
            n = int(np.prod(shape))
            self.offsets[name] = (off, n, tuple(shape))
            off = _align4(off + n)
        self.numel = off
        self.flat = torch.zeros(off, dtype=torch.float32, device=self.device)
        _register(self, self.flat)
        self.views = self._views(self.flat)
        self._grad = None
        self.m = None
        self.v = None
        self._seen = self.flat._version
        if init is not None:
            self.load_state_dict(init)

    def sync(self):
        """Announce torch-side writes to libaz_hip.so before the weights are read again.  The
        library caches fp16 planes of registered weights (az_weights_register) until
        az_weights_changed(); a write through a state_dict() / parameters() / params[k] view
        (an optimizer step, an in-place edit) would otherwise be served the OLD weights' planes.
        Every such write bumps the flat buffer's version counter (views share it), so comparing
        it with the one seen at the last sync finds them; every forward entry point calls this
        (one attribute read when nothing changed).  Writes by the library's own kernels
        (az_adam_f32) announce themselves.  Not seen: writes through `.data` and collectives
        that write parameter views in place (dist.broadcast / all_reduce) leave the version
        counter alone -- such a path calls weights_changed() (or copy_flat_) itself."""
        v = self.flat._version
        if v != self._seen:
            weights_changed()
            self._seen = v

    def _views(self, buf):
        return OrderedDict((k, buf[o:o + n].view(s)) for k, (o, n, s) in self.offsets.items())

    def __getitem__(self, k):
        return self.views[k]

    def span(self, prefix):
        """[start, end) of the flat buffer holding every tensor whose name starts with `prefix`
        (contiguous: tensors are laid out in spec order), e.g. "output_transform."."""
        hits = [(o, n) for k, (o, n, _) in self.offsets.items() if k.startswith(prefix)]
        if not hits:
            raise KeyError(prefix)
        s, e = hits[0][0], _align4(hits[-1][0] + hits[-1][1])
        if sum(_align4(n) for _, n in hits) != e - s:
            raise ValueError(f"tensors under {prefix!r} are not contiguous")
        return s, e

    def keys(self):
        return self.views.keys()

    # -- state_dict compatibility (torch.nn.Module semantics the reference relies on) --------
    def state_dict(self):
        return OrderedDict((k, v.detach()) for k, v in self.views.items())

    def cpu_state_dict(self):
        return OrderedDict((k, v.detach().cpu().clone()) for k, v in self.views.items())

    def load_state_dict(self, sd, strict=True):
        missing = [k for k in self.views if k not in sd]
        unexpected = [k for k in sd if k not in self.views]
        if strict and (missing or unexpected):
            raise RuntimeError(f"Error(s) in loading state_dict: missing keys {missing}, "
                               f"unexpected keys {unexpected}")
        for k, dst in self.views.items():
            if k not in sd:
                continue
            src = sd[k]
            if isinstance(src, np.ndarray):
                src = torch.from_numpy(np.ascontiguousarray(src))
            if tuple(src.shape) != tuple(dst.shape):
                raise RuntimeError(f"size mismatch for {k}: copying a param with shape "
                                   f"{tuple(src.shape)}, the shape in current model is "
                                   f"{tuple(dst.shape)}")
            dst.copy_(src.to(torch.float32), non_blocking=False)
        weights_changed()
        self._seen = self.flat._version

    def copy_flat_(self, src):
        """Overwrite the whole parameter buffer (a snapshot restore) and say so to the library."""
        self.flat.copy_(src)
        weights_changed()
        self._seen = self.flat._version

    # -- training buffers -------------------------------------------------------------------
    @property
    def grad_flat(self):
        if self._grad is None:
            self._grad = torch.zeros_like(self.flat)
            self.grads = self._views(self._grad)
        return self._grad

    def zero_grad(self):
        self.grad_flat.zero_()

    def reset_adam(self):
        """A fresh torch.optim.Adam (the reference builds one per train() call,
        Connect4GNN.py:132-133): zero moments, step count 0."""
        if self.m is None:
            self.m = torch.zeros_like(self.flat)
            self.v = torch.zeros_like(self.flat)
        else:
            self.m.zero_()
            self.v.zero_()
        self.step = 0
