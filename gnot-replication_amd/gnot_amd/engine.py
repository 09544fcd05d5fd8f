"""Host-side owner of one `gnot_plan`: parameters, batch geometry, workspace, grads.

All device memory is a torch tensor (the PyTorch caching allocator owns it); the native library
only receives pointers.  Kernel launches go on torch's current HIP stream.
"""
import ctypes
import itertools
import weakref

import torch

from . import _lib


def _ptr_array(ptrs):
    return (ctypes.c_void_p * len(ptrs))(*ptrs)


class Engine:
    def __init__(self, cfg: dict, linears):
        """cfg: the 12 constructor arguments; linears: nn.Linear modules in state_dict order."""
        self.lib = _lib.load()
        c = _lib.GnotConfig(**cfg)
        plan = ctypes.c_void_p()
        _lib.check(self.lib.gnot_plan_create(ctypes.byref(c), ctypes.byref(plan)))
        self.plan = plan
        n = self.lib.gnot_plan_num_linears(plan)
        dims = (ctypes.c_int32 * (2 * n))()
        _lib.check(self.lib.gnot_plan_linear_dims(plan, dims))
        self.dims = [(dims[2 * i], dims[2 * i + 1]) for i in range(n)]
        if len(linears) != n:
            raise RuntimeError(f"expected {n} Linears, module has {len(linears)}")
        for (o, i), lin in zip(self.dims, linears):
            if tuple(lin.weight.shape) != (o, i):
                raise RuntimeError(f"Linear shape {tuple(lin.weight.shape)} != plan {(o, i)}")
        self.linears = list(linears)
        self._bound_ptrs = None
        self.geom = None
        self.ws = None
        self.grad_views = None
        self.grad_arena = None     # flat fp32 view of every parameter gradient (one buffer)
        self.grad_hook = None      # optional callable(grad_arena) run after the backward kernels
        self.grad_flat = None      # the flat copy of the arena handed to autograd by the last backward
        self.param_grads = True    # False: no .grad tensors; grad_flat IS the arena (FlatAdamW reads it)
        self.comm = None           # parallel.PointShardComm when points are sharded over ranks
        self.grad_comm = None      # parallel.PointShardComm: gradients summed over ranks inside the backward
        self.moe_recompute = False # re-run each MoE call's expert forward in the backward (memory option)
        self.bf16 = False          # bf16 arithmetic mode of the MFMA kernels up to d = 256 (gnot_plan_set_precision)
        self.input_grads = False   # also differentiate x, theta, input functions (gnot_plan_set_input_grads)
        self.fwd_token = 0
        self.pending = None        # weakref to the autograd node of a training forward awaiting its backward
        self.pending_seq = 0

    _seq = itertools.count(1)

    def busy(self):
        """True while a training forward's backward is pending on this engine's activations."""
        return self.pending is not None and self.pending() is not None

    def mark_pending(self, node):
        self.pending = weakref.ref(node) if node is not None else None
        self.pending_seq = next(Engine._seq)

    def __del__(self):
        try:
            if getattr(self, "plan", None):
                self.lib.gnot_plan_destroy(self.plan)
        except Exception:
            pass

    # ---------------------------------------------------------------- binding
    def _bind_params(self):
        ws = [lin.weight for lin in self.linears]
        bs = [lin.bias for lin in self.linears]
        for t in ws + bs:
            if t.dtype in (torch.bfloat16, torch.float16):
                # the reference's bf16 route (module cast / autocast) is the bf16 arithmetic mode here, on fp32
                # parameters
                raise RuntimeError(f"gnot_amd parameters must stay float32 (got {t.dtype}): keep the module in "
                                   "fp32 and call set_precision('bf16') for bf16 arithmetic")
            if t.dtype == torch.float64:
                raise RuntimeError("gnot_amd computes in fp32 on the MFMA path; float64 modules are not supported "
                                   "(the fp64 restatement is oracle/gnot_oracle.py, test infrastructure)")
            if not (t.is_cuda and t.dtype == torch.float32 and t.is_contiguous()):
                raise RuntimeError("gnot_amd parameters must be contiguous float32 on a ROCm GPU")
        ptrs = tuple(t.data_ptr() for t in ws + bs)
        if ptrs != self._bound_ptrs:
            n = len(ws)
            _lib.check(self.lib.gnot_plan_bind_params(self.plan, _ptr_array(ptrs[:n]), _ptr_array(ptrs[n:])))
            self._bound_ptrs = ptrs
            self.geom = None   # workspace tables embed parameter pointers: rebind

    def prepare(self, x_off, fn_offs, training, device, n_global=None):
        """Set batch geometry (host int lists) and (re)bind the workspace when it changed.
        n_global: per-sample global point counts when the points are sharded over ranks (self.comm)."""
        self._bind_params()
        geom = (tuple(x_off), tuple(tuple(o) for o in fn_offs), bool(training),
                tuple(n_global) if n_global is not None else None, bool(self.moe_recompute), bool(self.bf16),
                bool(self.input_grads) and bool(training), id(self.grad_comm))
        if geom == self.geom:
            return
        B = len(x_off) - 1
        if self.comm is None and n_global is not None:
            raise ValueError("n_global was given but no point-shard communicator is set "
                             "(GNOT.set_point_shard): the local slice would be run as a whole mesh")
        if self.comm is not None:
            if n_global is None or len(n_global) != B:
                raise ValueError("point-sharded GNOT needs n_global (global points of every sample)")
            ng = (ctypes.c_int64 * B)(*[int(n) for n in n_global])
            _lib.check(self.lib.gnot_plan_set_shard(self.plan, self.comm.rank, self.comm.world, B, ng,
                                                    ctypes.byref(self.comm.struct)))
        else:
            _lib.check(self.lib.gnot_plan_set_shard(self.plan, 0, 1, 0, None, None))
        _lib.check(self.lib.gnot_plan_set_moe_recompute(self.plan, int(bool(self.moe_recompute))))
        _lib.check(self.lib.gnot_plan_set_precision(self.plan, int(bool(self.bf16))))
        _lib.check(self.lib.gnot_plan_set_input_grads(self.plan, int(bool(self.input_grads) and bool(training))))
        xo = (ctypes.c_int64 * (B + 1))(*x_off)
        flat = [v for o in fn_offs for v in o]
        fo = (ctypes.c_int64 * max(1, len(flat)))(*flat) if flat else None
        _lib.check(self.lib.gnot_plan_set_batch(self.plan, B, xo, fo, int(training)))
        need = self.lib.gnot_plan_workspace_bytes(self.plan)
        if self.ws is None or self.ws.numel() < need or self.ws.device != device:
            self.ws = None
            # 1/16 headroom: a stream of varying geometries (shuffled meshes) reuses one buffer
            self.ws = torch.empty(need + need // 16 + 256, dtype=torch.uint8, device=device)
        # stream-ordered table upload: no host synchronisation on a geometry change
        s = ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)
        _lib.check(self.lib.gnot_plan_bind_workspace_async(self.plan, self.ws.data_ptr(), self.ws.numel(), s))
        if self.comm is not None:
            self.comm.ws = self.ws
        if self.grad_comm is not None:
            self.grad_comm.ws = self.ws
            _lib.check(self.lib.gnot_plan_set_grad_comm(self.plan, ctypes.byref(self.grad_comm.struct)))
        else:
            _lib.check(self.lib.gnot_plan_set_grad_comm(self.plan, None))
        self.geom = geom
        self.grad_views = None
        self.grad_arena = None
        if training:
            n = len(self.dims)
            offs = (ctypes.c_int64 * (2 * n))()
            _lib.check(self.lib.gnot_plan_grad_offsets(self.plan, offs))
            base = self.debug_ptr("grads")[0] - self.ws.data_ptr()
            wsf = self.ws[: (self.ws.numel() // 4) * 4].view(torch.float32)
            views, layout = [], []
            for k, (o, i) in enumerate(self.dims):
                wo = base // 4 + offs[2 * k]
                bo = base // 4 + offs[2 * k + 1]
                views.append((wsf[wo:wo + o * i].view(o, i), wsf[bo:bo + o]))
                layout.append((offs[2 * k], offs[2 * k + 1], (o, i), o))
            self.grad_views = views
            self.grad_layout = layout          # offsets relative to the arena start
            last_o = self.dims[-1][0]
            self.grad_arena = wsf[base // 4: base // 4 + offs[2 * n - 1] + last_o]

    def debug_ptr(self, name):
        ptr = ctypes.c_void_p()
        ld = ctypes.c_int64()
        _lib.check(self.lib.gnot_debug_buffer(self.plan, name.encode(), ctypes.byref(ptr), ctypes.byref(ld)))
        return ptr.value, ld.value

    def debug_tensor(self, name, rows, cols):
        """Copy of a named workspace buffer as a [rows, cols] float32 tensor (tests / debugging)."""
        ptr, ld = self.debug_ptr(name)
        off = (ptr - self.ws.data_ptr()) // 4
        wsf = self.ws[: (self.ws.numel() // 4) * 4].view(torch.float32)
        ld = ld if ld > 0 else cols
        return wsf[off:off + rows * ld].view(rows, ld)[:, :cols].clone()

    def profile_enable(self, kind):
        _lib.check(self.lib.gnot_profile_enable(self.plan, (kind or "").encode()))

    def profile_read(self):
        """(device ms summed over launches, launches, algorithmic FLOPs) since enable/last read."""
        ms, n, fl = ctypes.c_double(), ctypes.c_int64(), ctypes.c_double()
        _lib.check(self.lib.gnot_profile_read(self.plan, ctypes.byref(ms), ctypes.byref(n), ctypes.byref(fl)))
        return ms.value, n.value, fl.value

    # ---------------------------------------------------------------- compute
    def stream(self):
        """torch's current stream ON THE WORKSPACE'S DEVICE (not the current device's)."""
        return ctypes.c_void_p(torch.cuda.current_stream(self.ws.device).cuda_stream)

    def _own_comms(self):
        """the communicators view raw pointers through ONE workspace tensor: this engine's, for its calls
        (another engine of the same module may have been prepared since)"""
        for c in (self.comm, self.grad_comm):
            if c is not None:
                c.ws = self.ws

    def forward(self, x, theta, fns, out):
        self._own_comms()
        s = self.stream()
        _lib.check(self.lib.gnot_pack_weights(self.plan, s))
        fptr = _ptr_array([f.data_ptr() for f in fns]) if fns else None
        _lib.check(self.lib.gnot_forward(self.plan, x.data_ptr(), theta.data_ptr(), fptr, out.data_ptr(), s))
        self.fwd_token += 1
        return self.fwd_token

    def input_grads_into(self, dx, dtheta, dfns):
        """Gradients of x [P, in], theta [B, th] and the input functions [Q_i, F] of the last backward
        (None entries are skipped); launched on torch's current stream."""
        ptr = lambda t: t.data_ptr() if t is not None else None
        fptr = _ptr_array([ptr(f) for f in dfns]) if dfns else None
        self._own_comms()
        with torch.cuda.device(self.ws.device):
            _lib.check(self.lib.gnot_input_grads(self.plan, ptr(dx), ptr(dtheta), fptr, self.stream()))

    def backward(self, dout):
        self._own_comms()
        with torch.cuda.device(self.ws.device):
            _lib.check(self.lib.gnot_backward(self.plan, dout.data_ptr(), self.stream()))
        if self.grad_hook is not None:
            self.grad_hook(self.grad_arena)     # e.g. ONE all-reduce of all gradients (sample-DP)
        return self.grad_views
