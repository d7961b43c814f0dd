"""Batched solve context: the Python face of ``vc_ctx`` (include/vcmpc.h).

Every method takes either host numpy arrays (the call stages them through the
context's device arena and returns when results are back in the caller's arrays)
or device-resident ``torch`` tensors on the context's GPU (the call only enqueues
work on the context stream -- the fast path, used by ``bench.py``).

Shapes (batch-outermost, C-contiguous, state/action orders of the reference
FancyVector keys, see include/vcmpc.h):

    x0[B, nx]  kappa[B, N]  ds[B, N]  ubar[B, N, nu]  xbar[B, NS, nx]  u0[B, nu]

NS = N + 1 state columns for the kinematic model (kinematic_mpc.py:59), N for the
dynamic single-track model (cascaded_mpc.py:70); vc_rollout / vc_linearize use N + 1.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _abi
from .config import make_params

NX = {_abi.VC_MODEL_KINEMATIC: 6, _abi.VC_MODEL_DYNAMIC: 8, _abi.VC_MODEL_CASCADED: 8}
NU = 2
_NP_DT = {_abi.VC_F64: np.float64, _abi.VC_F32: np.float32}


def _is_torch(a) -> bool:
    return type(a).__module__.startswith("torch")


class Context:
    """One solve context (one device, one model, one horizon, one stream)."""

    def __init__(self, model: int = _abi.VC_MODEL_KINEMATIC, N: int = 20, max_batch: int = 1024,
                 dtype: int = _abi.VC_F64, device: int = 0, params: _abi.vc_params | None = None, **cfgs):
        self.lib = _abi.load_library()
        self.model, self.N, self.max_batch, self.dtype, self.device = model, int(N), int(max_batch), dtype, device
        self.nx = NX[model]
        self.params = params if params is not None else make_params(**cfgs)
        # stages of the solve arrays: N + 1 states (kinematic), N (single track), or
        # H = N + horizon_pm (cascaded: kappa, ds, ubar, xbar span the point-mass tail too)
        self.NH = self.N + (int(self.params.casc.horizon_pm) if model == _abi.VC_MODEL_CASCADED else 0)
        self.ns_solve = self.N + 1 if model == _abi.VC_MODEL_KINEMATIC else self.NH
        h = self.lib.vc_create(device, model, self.N, self.max_batch, dtype, C.byref(self.params))
        if not h:
            raise _abi.VcError(_abi.VC_E_HIP, self.lib.vc_last_error(None).decode())
        self._h = C.c_void_p(h)

    # -- lifetime ---------------------------------------------------------------
    def close(self):
        if getattr(self, "_h", None):
            self.lib.vc_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def _check(self, code):
        _abi.check(self.lib, self._h, code)

    def set_stream(self, stream_handle: int | None):
        """Run on an external HIP stream (e.g. ``torch.cuda.current_stream().cuda_stream``)."""
        self._check(self.lib.vc_set_stream(self._h, C.c_void_p(stream_handle or 0)))

    def set_obstacles(self, obstacles, margin_min: float = 0.0):
        """``vc_set_obstacles``: replace the obstacle list [(s, ey, radius), ...] the
        barrier terms use (Track._construct_obstacles, track.py:131-138); [] = off."""
        rows = np.asarray([tuple(r) for r in (obstacles or [])], np.float64).reshape(-1, 3)
        cols = [np.ascontiguousarray(rows[:, i]) for i in range(3)]
        self._check(self.lib.vc_set_obstacles(self._h, len(rows), *[C.c_void_p(c.ctypes.data) for c in cols],
                                              float(margin_min)))

    def synchronize(self):
        self._check(self.lib.vc_synchronize(self._h))

    # -- argument marshalling -----------------------------------------------------
    def _marshal(self, arrays, shapes, dtypes):
        """Validate a set of buffers; all host numpy or all device torch.
        Returns (pointers, flags)."""
        dev = [_is_torch(a) for a in arrays]
        if any(dev) and not all(dev):
            raise TypeError("mix of host and device buffers in one call")
        ptrs = []
        for a, shp, dt in zip(arrays, shapes, dtypes):
            if dev[0]:
                import torch
                tdt = {np.float64: torch.float64, np.float32: torch.float32, np.int32: torch.int32}[dt]
                if a.dtype != tdt or not a.is_contiguous() or tuple(a.shape) != tuple(shp):
                    raise ValueError(f"device buffer must be contiguous {tdt}{tuple(shp)}, got {a.dtype}{tuple(a.shape)}")
                if not a.is_cuda or a.device.index != self.device:
                    raise ValueError(f"device buffer must live on cuda:{self.device}")
                ptrs.append(C.c_void_p(a.data_ptr()))
            else:
                if not isinstance(a, np.ndarray) or a.dtype != dt or not a.flags.c_contiguous or a.shape != tuple(shp):
                    got = f"{getattr(a, 'dtype', type(a))}{getattr(a, 'shape', '')}"
                    raise ValueError(f"host buffer must be C-contiguous {np.dtype(dt)}{tuple(shp)}, got {got}")
                ptrs.append(C.c_void_p(a.ctypes.data))
        return ptrs, (_abi.VC_DEVICE_PTRS if dev[0] else _abi.VC_HOST_PTRS)

    def _batch(self, x):
        B = int(x.shape[0])
        if B > self.max_batch:
            raise ValueError(f"batch {B} > max_batch {self.max_batch}")
        return B

    # -- entry points -------------------------------------------------------------
    def solve(self, x0, kappa, ds, ubar, xbar=None, u0=None, status=None, iters=None, diag=None):
        """One MPC step (``vc_solve``: LTV-QP for the kinematic model, SQP for the
        dynamic one).  ``ubar`` is the warm start and is
        overwritten with u*; returns (u0, xbar, ubar, status, iters).  With
        ``diag=True`` (or a [B, 4] buffer) it calls ``vc_solve_diag`` and returns
        the per-problem solver diagnostics as a sixth element."""
        B, N, nx, f = self._batch(x0), self.NH, self.nx, _NP_DT[self.dtype]
        NS = self.ns_solve
        if xbar is None and self.model == _abi.VC_MODEL_KINEMATIC and self.params.qp.ms:
            raise ValueError("vc_qp.ms: multiple shooting linearises at the state iterate; pass xbar")
        if _is_torch(x0):
            import torch
            kw = dict(device=x0.device)
            xbar = torch.empty((B, NS, nx), dtype=x0.dtype, **kw) if xbar is None else xbar
            u0 = torch.empty((B, NU), dtype=x0.dtype, **kw) if u0 is None else u0
            status = torch.empty((B,), dtype=torch.int32, **kw) if status is None else status
            iters = torch.empty((B,), dtype=torch.int32, **kw) if iters is None else iters
        else:
            xbar = np.empty((B, NS, nx), f) if xbar is None else xbar
            u0 = np.empty((B, NU), f) if u0 is None else u0
            status = np.empty((B,), np.int32) if status is None else status
            iters = np.empty((B,), np.int32) if iters is None else iters
        bufs = [x0, kappa, ds, xbar, ubar, u0, status, iters]
        shapes = [(B, nx), (B, N), (B, N), (B, NS, nx), (B, N, NU), (B, NU), (B,), (B,)]
        dts = [f, f, f, f, f, f, np.int32, np.int32]
        if diag is not None and diag is not False:
            if diag is True:
                diag = self._like(x0, (B, 4))
            # [B, 4]; timing builds (libvcmpc_timing.so) append section-cycle columns
            ptrs, flags = self._marshal(bufs + [diag], shapes + [(B, int(diag.shape[1]))], dts + [f])
            self._check(self.lib.vc_solve_diag(self._h, B, *ptrs, flags))
            return u0, xbar, ubar, status, iters, diag
        ptrs, flags = self._marshal(bufs, shapes, dts)
        self._check(self.lib.vc_solve(self._h, B, *ptrs, flags))
        return u0, xbar, ubar, status, iters

    def solve_from(self, x0, kappa, ds, ubar_in, u_out, xbar=None, u0=None, status=None, iters=None):
        """``vc_solve_from``: ``solve`` with the warm start read from ``ubar_in``, which is left
        unchanged, and u* written to ``u_out``; returns (u0, xbar, u_out, status, iters)."""
        B, N, nx, f = self._batch(x0), self.NH, self.nx, _NP_DT[self.dtype]
        NS = self.ns_solve
        if xbar is None and self.model == _abi.VC_MODEL_KINEMATIC and self.params.qp.ms:
            raise ValueError("vc_qp.ms: multiple shooting linearises at the state iterate; pass xbar")
        if _is_torch(x0):
            import torch
            kw = dict(device=x0.device)
            xbar = torch.empty((B, NS, nx), dtype=x0.dtype, **kw) if xbar is None else xbar
            u0 = torch.empty((B, NU), dtype=x0.dtype, **kw) if u0 is None else u0
            status = torch.empty((B,), dtype=torch.int32, **kw) if status is None else status
            iters = torch.empty((B,), dtype=torch.int32, **kw) if iters is None else iters
        else:
            xbar = np.empty((B, NS, nx), f) if xbar is None else xbar
            u0 = np.empty((B, NU), f) if u0 is None else u0
            status = np.empty((B,), np.int32) if status is None else status
            iters = np.empty((B,), np.int32) if iters is None else iters
        bufs = [x0, kappa, ds, ubar_in, xbar, u_out, u0, status, iters]
        shapes = [(B, nx), (B, N), (B, N), (B, N, NU), (B, NS, nx), (B, N, NU), (B, NU), (B,), (B,)]
        dts = [f, f, f, f, f, f, f, np.int32, np.int32]
        ptrs, flags = self._marshal(bufs, shapes, dts)
        self._check(self.lib.vc_solve_from(self._h, B, *ptrs, flags))
        return u0, xbar, u_out, status, iters

    def solve_debug(self, x0, kappa, ds, ubar):
        """``vc_solve_debug`` (dynamic contexts): the solve plus a dump of the first
        QP's internals (g, normal matrix, factor storage, predictor rhs and step)."""
        B, N, nx, f = self._batch(x0), self.N, self.nx, np.float32
        stride = self.lib.vc_debug_stride()
        xbar, u0 = np.empty((B, self.ns_solve, nx), f), np.empty((B, NU), f)
        status, iters, dbg = np.empty(B, np.int32), np.empty(B, np.int32), np.empty((B, stride), f)
        ptrs, flags = self._marshal([x0, kappa, ds, xbar, ubar, u0, status, iters, dbg],
                                    [(B, nx), (B, N), (B, N), (B, self.ns_solve, nx), (B, N, NU), (B, NU), (B,),
                                     (B,), (B, stride)], [f] * 6 + [np.int32, np.int32, f])
        self._check(self.lib.vc_solve_debug(self._h, B, *ptrs, flags))
        n = 2 * N
        return dict(u0=u0, xbar=xbar, ubar=ubar, status=status, iters=iters, g=dbg[:, :n],
                    M=dbg[:, n:n + n * n].reshape(B, n, n), Y=dbg[:, n + n * n:n + 2 * n * n].reshape(B, n, n),
                    rhs=dbg[:, n + 2 * n * n:2 * n + 2 * n * n], dz=dbg[:, 2 * n + 2 * n * n:3 * n + 2 * n * n])

    def rollout(self, x0, ubar, kappa, ds):
        B, N, nx, f = self._batch(x0), self.N, self.nx, _NP_DT[self.dtype]
        xbar = self._like(x0, (B, N + 1, nx))
        ptrs, flags = self._marshal([x0, ubar, kappa, ds, xbar],
                                    [(B, nx), (B, N, NU), (B, N), (B, N), (B, N + 1, nx)], [f] * 5)
        self._check(self.lib.vc_rollout(self._h, B, *ptrs, flags))
        return xbar

    def linearize(self, xbar, ubar, kappa, ds):
        B, N, nx, f = self._batch(xbar), self.N, self.nx, _NP_DT[self.dtype]
        A = self._like(xbar, (B, N, nx, nx))
        Bm = self._like(xbar, (B, N, nx, NU))
        ptrs, flags = self._marshal([xbar, ubar, kappa, ds, A, Bm],
                                    [(B, N + 1, nx), (B, N, NU), (B, N), (B, N), (B, N, nx, nx), (B, N, nx, NU)],
                                    [f] * 6)
        self._check(self.lib.vc_linearize(self._h, B, *ptrs, flags))
        return A, Bm

    def condense(self, x0, ubar, kappa, ds):
        B, N, nx, f = self._batch(x0), self.NH, self.nx, _NP_DT[self.dtype]
        n = NU * N
        H = self._like(x0, (B, n, n))
        g = self._like(x0, (B, n))
        ptrs, flags = self._marshal([x0, ubar, kappa, ds, H, g],
                                    [(B, nx), (B, N, NU), (B, N), (B, N), (B, n, n), (B, n)], [f] * 6)
        self._check(self.lib.vc_condense(self._h, B, *ptrs, flags))
        return H, g

    def plant_step(self, x, u, kappa, dt):
        B, nx, f = self._batch(x), self.nx, _NP_DT[self.dtype]
        xn = self._like(x, (B, nx))
        px, pu, pk, pxn = self._marshal([x, u, kappa, xn], [(B, nx), (B, NU), (B,), (B, nx)], [f] * 4)[0]
        flags = _abi.VC_DEVICE_PTRS if _is_torch(x) else _abi.VC_HOST_PTRS
        self._check(self.lib.vc_plant_step(self._h, B, px, pu, pk, float(dt), pxn, flags))
        return xn

    def ode(self, x, u, kappa, space=False):
        """``vc_ode``: the model's vector field f(x, u, kappa) (temporal, or spatial with
        ``space=True``) for B points."""
        B, nx, f = self._batch(x), self.nx, _NP_DT[self.dtype]
        fo = self._like(x, (B, nx))
        ptrs, flags = self._marshal([x, u, kappa, fo], [(B, nx), (B, NU), (B,), (B, nx)], [f] * 4)
        p = ptrs
        self._check(self.lib.vc_ode(self._h, B, p[0], p[1], p[2], int(bool(space)), p[3], flags))
        return fo

    def spatial_step(self, x, u, kappa, ds):
        B, nx, f = self._batch(x), self.nx, _NP_DT[self.dtype]
        xn = self._like(x, (B, nx))
        ptrs, flags = self._marshal([x, u, kappa, ds, xn], [(B, nx), (B, NU), (B,), (B,), (B, nx)], [f] * 5)
        self._check(self.lib.vc_spatial_step(self._h, B, *ptrs, flags))
        return xn

    # -- track table and closed loop ----------------------------
    def set_track(self, track):
        """Upload ``track``'s curvature table (``vc_track_set``); ``track`` is a
        ``vcmpc.environment.Track`` (or anything with ``kappa_table()``)."""
        coef, h, length = track.kappa_table()
        coef = np.ascontiguousarray(coef, np.float64)
        self._check(self.lib.vc_track_set(self._h, int(coef.shape[0]), float(h), float(length),
                                          C.c_void_p(coef.ctypes.data)))
        self.track = track

    def track_k(self, s):
        B, f = self._batch(s), _NP_DT[self.dtype]
        k = self._like(s, (B,))
        ptrs, flags = self._marshal([s, k], [(B,), (B,)], [f, f])
        self._check(self.lib.vc_track_k(self._h, B, *ptrs, flags))
        return k

    def horizon(self, x0, xbar, mpc_dt):
        """``_init_horizon`` on the device: (kappa[B, N], ds[B, N]) from the state and
        the unshifted warm start xbar[B, NS, nx]."""
        B, N, nx, f = self._batch(x0), self.NH, self.nx, _NP_DT[self.dtype]
        kappa, ds = self._like(x0, (B, N)), self._like(x0, (B, N))
        ptrs, flags = self._marshal([x0, xbar, kappa, ds], [(B, nx), (B, self.ns_solve, nx), (B, N), (B, N)], [f] * 4)
        self._check(self.lib.vc_horizon(self._h, B, ptrs[0], ptrs[1], float(mpc_dt), ptrs[2], ptrs[3], flags))
        return kappa, ds

    def drive(self, x64, u0, dt, x_ctx=None):
        """``RacingCar.drive`` for B vehicles: x64[B, nx] (fp64) is advanced in place
        with k(s) from the track table; returns x64 (and fills x_ctx if given)."""
        B, nx, f = self._batch(x64), self.nx, _NP_DT[self.dtype]
        arrs, shapes, dts = [x64, u0], [(B, nx), (B, NU)], [np.float64, f]
        if x_ctx is not None:
            arrs, shapes, dts = arrs + [x_ctx], shapes + [(B, nx)], dts + [f]
        ptrs, flags = self._marshal(arrs, shapes, dts)
        xc = ptrs[2] if x_ctx is not None else None
        self._check(self.lib.vc_drive(self._h, B, ptrs[0], ptrs[1], float(dt), xc, flags))
        return x64

    def simulate(self, x64, xbar, ubar, steps, mpc_dt, dt, log=False, nfail=None):
        """``vc_simulate``: ``steps`` closed-loop steps (horizon -> solve -> drive) on the
        device.  x64, xbar, ubar are updated in place.  With ``log=True`` returns
        (log_x[steps+1, B, nx] fp64, log_u[steps, B, nu], nfail[B]); else (None, None, nfail)."""
        B, N, nx, f = self._batch(x64), self.NH, self.nx, _NP_DT[self.dtype]
        steps = int(steps)
        dev = _is_torch(x64)
        if nfail is None:
            if dev:
                import torch
                nfail = torch.zeros((B,), dtype=torch.int32, device=x64.device)
            else:
                nfail = np.zeros((B,), np.int32)
        arrs = [x64, xbar, ubar, nfail]
        shapes = [(B, nx), (B, self.ns_solve, nx), (B, N, NU), (B,)]
        dts = [np.float64, f, f, np.int32]
        log_x = log_u = None
        if log:
            if dev:
                import torch
                log_x = torch.empty((steps + 1, B, nx), dtype=torch.float64, device=x64.device)
                log_u = torch.empty((steps, B, NU), dtype=xbar.dtype, device=x64.device)
            else:
                log_x, log_u = np.empty((steps + 1, B, nx)), np.empty((steps, B, NU), f)
            arrs, shapes, dts = arrs + [log_x, log_u], shapes + [(steps + 1, B, nx), (steps, B, NU)], dts + [np.float64, f]
        ptrs, flags = self._marshal(arrs, shapes, dts)
        lx, lu = (ptrs[4], ptrs[5]) if log else (None, None)
        self._check(self.lib.vc_simulate(self._h, B, steps, float(mpc_dt), float(dt), ptrs[0], ptrs[1], ptrs[2],
                                         lx, lu, ptrs[3], flags))
        return log_x, log_u, nfail

    def _like(self, ref, shape):
        if _is_torch(ref):
            import torch
            return torch.empty(shape, dtype=ref.dtype, device=ref.device)
        return np.empty(shape, _NP_DT[self.dtype])
