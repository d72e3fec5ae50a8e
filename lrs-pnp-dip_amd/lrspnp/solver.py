"""Batched LRS-PnP ADMM outer loop on one MI355X (host orchestration only).

Mirrors the module-level loop of main_LRS_PnP.py:244-366 (SVT low-rank prox) with the DIP
variants' ISTA rule selectable (…1-LiP.py:185-198).  One `step()` = one outer ADMM iteration:

    main stream : im2col(X + L1/mu1) -> fused masked ISTA + PnP prox (all blocks) -> Phi
    lowrank str.: SVT(X + L2/mu2, 1/mu2) -> U            (runs concurrently with the ISTA)
    main stream : col2im + closed-form X + dual updates + ||delta||^2   (waits for both)

No per-block Python, no host synchronisation inside `step()`.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch

from . import ops
from ._lib import LrsError
from .dip import stream_wait


@dataclass
class LrsPnPConfig:
    """The knob table of SURVEY.md §5 (main_LRS_PnP.py:218-238 defaults)."""
    gamma: float = 0.5            # data fidelity                      main_LRS_PnP.py:218
    mu1: float = 0.15             # sparsity penalty                   :221
    mu2: float = 0.15 * 6         # low-rank penalty                   :222
    lambda_ista: float = 0.1      # ISTA lambda                         :225
    Nit: int = 80                 # inner ISTA iterations               :226
    bb: int = 36                  # block size                          :237
    sliding: int = 36             # slidingDis                          :238
    variant: str = "spec2"        # 'spec2' (main), 'fro4' (DIP mains), 'soft' (ista.m), 'matlab' (pnp_ista.m)
    svt_method: str = "tri"       # SVT eigensolver: 'tri' (tridiagonal, certified) or 'jacobi'
    svt_warm: bool = True         # warm-start the Jacobi eigensolver from the previous iteration
    svt_gram_first: bool = False  # hold the sparse coding until the SVT Gram is done (always for Jacobi)
    # The tridiagonal eigensolver's eigenvalue / inverse-iteration / back-transformation phases over
    # many workgroups (LRS_SVT_MULTI_WG, bit-identical): "auto" on a row-slab shard, where the
    # replicated solve is on the critical path; the one-workgroup chain beside a whole-cube sparse
    # coding (a multi-launch chain there waits for free CUs between its launches).
    svt_multi_wg: str = "auto"
    lowrank: str = "svt"          # 'svt' (main_LRS_PnP.py:315) or 'dip' (…1-LiP.py:399-411)
    dip: object = None            # lrspnp.dip.DipConfig for lowrank='dip' (None: reference defaults)
    dip_seed: int = 0             # DIP init seed of outer iteration t is dip_seed + t
    # Workgroups of the sparse-coding kernel beside the DIP training (lowrank='dip';
    # lrs_ista_opts.max_workgroups, 0 = one per 16-block tile).  Measured at configs[2]
    # (bench.py --ista-max-wg): 0 -> 7.25 outer it/s, 128 -> 7.18, 64 -> 6.97, 32 -> 6.68: a longer,
    # narrower sparse coding taxes the DIP more than a short full-chip one, so unbounded.  Re-measured
    # on the per-pattern kernel (405 tiles, 3 interleaved rounds, profiles/r04/ista_max_wg/):
    # 0 -> 7.85 / 7.84 / 7.84, 256 -> 7.84 / 7.84 / 7.82, 128 -> 7.80 / 7.81 / 7.80.
    ista_max_wg_dip: int = 0
    # Launches the sparse coding's Nit iterations are split over beside the DIP training
    # (lowrank='dip'; lrs_ista_opts.warm_start: the iterates are exactly those of one launch).  A
    # workgroup of one launch holds its CU for the whole Nit; slices free CUs for the DIP's kernels
    # every Nit / slices iterations.  Measured at configs[2] (bench.py --ista-slices, 2 rounds):
    # 1 -> 7.50 outer it/s, 4 -> 7.49, 10 -> 7.39-7.42, 25 -> 7.27 (each slice re-forms D^T(m.*y) and
    # Phi, and runs longer beside the DIP than its share of one launch), so one launch.
    ista_slices_dip: int = 1
    # Priority of the low-rank stream (torch.cuda.Stream priority: 0 = default, negative = higher).
    # Beside the DIP, the sparse-coding kernel's resident workgroups can hold off a 1024-thread
    # BatchNorm workgroup of the DIP for milliseconds; a higher-priority queue asks the dispatcher to
    # place the DIP's workgroups first.  Measured at configs[2] (bench.py --lowrank-priority, 2
    # alternating rounds): 0 -> 7.43 / 7.43 outer it/s, -1 -> 7.48 / 7.41: no effect, so 0.
    lowrank_priority: int = 0
    # Order of the sparse coding and the DIP training (lowrank='dip'): "beside" runs the
    # sparse-coding kernel concurrently with the DIP's first steps; "before" makes the DIP's stream
    # wait for it (the kernel then has the chip to itself).
    ista_dip_order: str = "beside"
    # Sparse coding on per-pattern masked Grams (lrs_ista_pat_f32: the blocks grouped by observation
    # pattern, 2 K^2 instead of 4 n K FLOP per block and iteration): "auto" when the library's cost
    # model prefers it (few patterns, n > K / 2), "on" whenever the block length allows it, "off".
    ista_patterns: str = "auto"

    @staticmethod
    def dip_1lip(**kw) -> "LrsPnPConfig":
        """Parameters of main_LRS_PnP_DIP_1-LiP.py:316-345: fro4 ISTA (Nit 100), mu1 = mu2 = 0.1,
        and the 1-Lipschitz U-Net DIP as the low-rank prox."""
        base = dict(gamma=0.5, mu1=0.1, mu2=0.1, lambda_ista=0.1, Nit=100, bb=36, sliding=36, variant="fro4",
                    lowrank="dip")
        base.update(kw)
        return LrsPnPConfig(**base)

    @staticmethod
    def dip_pro(**kw) -> "LrsPnPConfig":
        """main_LRS_PnP_DIP_pro.py:324-353: as dip_1lip, with the skip() network (5 scales of 128
        channels, 128-channel skips, plain BatchNorm, Sigmoid) as the DIP prox (:215-221)."""
        from .dip import DipConfig
        dip = kw.pop("dip", None) or DipConfig(net="skip")
        if dip.net != "skip":
            raise LrsError("dip_pro uses the skip network")
        base = dict(gamma=0.5, mu1=0.1, mu2=0.1, lambda_ista=0.1, Nit=100, bb=36, sliding=36, variant="fro4",
                    lowrank="dip", dip=dip)
        base.update(kw)
        return LrsPnPConfig(**base)


_ALPHA = {"spec2": ops.ALPHA_SPEC2, "fro4": ops.ALPHA_FRO4, "soft": ops.ALPHA_SOFT, "matlab": ops.ALPHA_SPEC2}
_PROX = {"spec2": ops.PROX_NLM, "fro4": ops.PROX_NLM, "soft": ops.PROX_SOFT, "matlab": ops.PROX_NLM_MATLAB}


class LrsPnP:
    """LRS-PnP solver state on the current ROCm device.

    Y: observed unfolded cube (P x B, zeros at missing entries), M: mask (P x B), D: n x K
    dictionary with n = bb*bb.  All float32 (numpy or torch); copied to the device once.
    """

    def __init__(self, Y, M, D, cfg: LrsPnPConfig | None = None, device="cuda", image_shape=None, comm=None,
                 dip_engine: bool = True):
        """dip_engine=False (lowrank='dip' only): keep the DIP's target / mask / U buffers but build
        no network engine -- a task-parallel worker rank that never trains the DIP
        (lrspnp.dist.DipTaskSplit)."""
        self.cfg = cfg = cfg or LrsPnPConfig()
        # comm: None (whole cube here) or a row-slab communicator (lrspnp.dist.SlabComm): Y, M are
        # then this rank's pixel-row slab and the SVT Gram / convergence sums are all-reduced
        self.comm = comm
        dev = torch.device(device)
        f = lambda a: torch.as_tensor(np.asarray(a, np.float32) if not isinstance(a, torch.Tensor) else a,
                                      dtype=torch.float32).to(dev).contiguous()
        self.Y, self.M, self.D = f(Y), f(M), f(D)
        self.P, self.B = self.Y.shape
        n, self.K = self.D.shape
        if n != cfg.bb * cfg.bb:
            raise LrsError(f"dictionary has {n} rows, expected bb*bb = {cfg.bb * cfg.bb}")
        self.n = n
        self.n_pad = -(-n // 16) * 16
        f32 = np.float32
        self.gamma32, self.mu1_32, self.mu2_32 = f32(cfg.gamma), f32(cfg.mu1), f32(cfg.mu2)
        self.c2 = f32(1 / cfg.mu2)                        # (1/mu_2)*lambda_2   main_LRS_PnP.py:315
        self.tau = float(f32(1 / cfg.mu2))                # SVT threshold (float32 in numpy)
        if cfg.variant not in _PROX:
            raise LrsError(f"unknown ISTA variant {cfg.variant!r} (spec2 | fro4 | soft | matlab)")
        self.prox = _PROX[cfg.variant]

        # ---- block grid (host bookkeeping) -------------------------------------------------
        rows, cols = ops.block_grid(self.P, self.B, cfg.bb, cfg.sliding)
        self.nb = rows.size
        rstarts = np.unique(rows).astype(np.int32)
        cstarts = np.unique(cols).astype(np.int32)
        self.nbr = rstarts.size
        assert np.array_equal(rows, np.tile(rstarts, cstarts.size))
        assert np.array_equal(cols, np.repeat(cstarts, rstarts.size))
        rlo, rhi = ops.cover_ranges(self.P, cfg.bb, rstarts)
        clo, chi = ops.cover_ranges(self.B, cfg.bb, cstarts)
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
        self.rows_d, self.cols_d = t(rows), t(cols)
        self.grid = dict(rstarts=t(rstarts), cstarts=t(cstarts), nbr=self.nbr, rlo=t(rlo), rhi=t(rhi),
                         clo=t(clo), chi=t(chi))

        # ---- observation masks of blocks_copy (main_LRS_PnP.py:244,278) and alpha/h --------
        _, obs = ops.im2col(self.Y, None, 1.0, cfg.bb, self.rows_d, self.cols_d, self.n_pad, want_obs=True)
        self.obs = obs
        packed = np.packbits(obs.cpu().numpy(), axis=1)
        uniq, inv = np.unique(packed, axis=0, return_inverse=True)
        self.npat = uniq.shape[0]
        obs_pat = t(np.unpackbits(uniq, axis=1)[:, : self.n_pad].astype(np.uint8))
        alpha_pat, thr_pat = ops.ista_alpha(self.D, obs_pat, n, _ALPHA[cfg.variant], cfg.lambda_ista)
        inv_d = t(inv.reshape(-1).astype(np.int64))
        self.alpha = alpha_pat.index_select(0, inv_d).contiguous()
        self.thr = thr_pat.index_select(0, inv_d).contiguous()
        self.alpha_pat, self.thr_pat, self.obs_pat = alpha_pat, thr_pat, obs_pat
        self.pat_plan = None
        if cfg.ista_patterns not in ("auto", "on", "off"):
            raise LrsError(f"unknown ista_patterns {cfg.ista_patterns!r} (auto | on | off)")
        # every mode string is checked here, before anything is enqueued (not halfway through step())
        if cfg.ista_dip_order not in ("beside", "before"):
            raise LrsError(f"unknown ista_dip_order {cfg.ista_dip_order!r} (beside | before)")
        if cfg.svt_multi_wg not in ("auto", "on", "off"):
            raise LrsError(f"unknown svt_multi_wg {cfg.svt_multi_wg!r} (auto | on | off)")
        if self.K <= 512 and (cfg.ista_patterns == "on" or (
                cfg.ista_patterns == "auto" and ops.ista_pat_preferred(n, self.K, self.nb, self.npat, cfg.Nit))):
            plan, self.pat_ntiles = ops.ista_pat_plan(inv.reshape(-1), self.npat)
            self.pat_plan = t(plan)

        # ---- state and buffers -------------------------------------------------------------
        self.X = self.Y.clone()                           # X = Y_observed     main_LRS_PnP.py:229
        self.L1 = torch.zeros_like(self.Y)
        self.L2 = torch.zeros_like(self.Y)
        self.U = torch.empty_like(self.Y)
        self.Yb = torch.empty((self.nb, self.n_pad), dtype=torch.float32, device=dev)
        self.phi = torch.empty((self.nb, self.n_pad), dtype=torch.float32, device=dev)
        if self.pat_plan is not None:   # the dictionary and Gram images, once per solve (D, patterns fixed)
            self.ista_ws = ops.ista_pat_prepare(self.D, self.obs_pat, n)
        else:
            self.ista_ws = ops.ista_workspace(n, self.K, self.prox, dev)
        self.norms = torch.zeros(3, dtype=torch.float64, device=dev)
        self.lowrank_stream = torch.cuda.Stream(device=dev, priority=int(cfg.lowrank_priority))
        self.iteration = 0
        self.dip = None
        if comm is not None and (cfg.lowrank != "svt" or cfg.svt_method != "tri"):
            raise LrsError("a row-slab shard needs lowrank='svt' with svt_method='tri'")
        if cfg.lowrank == "svt":
            self.svt_ws = ops.svt_workspace(self.P, self.B, dev)
            self.gram = ops.svt_gram_view(self.svt_ws, self.P, self.B) if comm is not None else None
        elif cfg.lowrank == "dip":
            self._init_dip(image_shape, dev, engine=dip_engine)
        else:
            raise LrsError(f"unknown lowrank prox {cfg.lowrank!r}")

    def _init_dip(self, image_shape, dev, engine=True):
        """DIP target = the observed cube as an image, mask_bkg = the pixel mask
        (…1-LiP.py:275-301); the network is re-initialised every outer iteration (:214)."""
        from .dip import DipConfig, LipschitzDip
        if image_shape is None:
            raise LrsError("lowrank='dip' needs image_shape=(H, W) with H*W = P")
        H, W = (int(v) for v in image_shape)
        if H * W != self.P:
            raise LrsError(f"image_shape {H}x{W} does not match P = {self.P}")
        self.H, self.W = H, W
        self.dip = LipschitzDip(self.B, H, W, self.cfg.dip or DipConfig(), device=dev,
                                 stream_priority=self.cfg.lowrank_priority) if engine else None
        self.dip_target = torch.empty((self.B, H, W), dtype=torch.float32, device=dev)
        ops.unfolded_to_image(self.Y, None, 1.0, H, W, self.dip_target)
        pix = ops.unfolded_to_image(self.M[:, :1].contiguous(), None, 1.0, H, W)   # (1, H, W)
        self.dip_mask = pix.reshape(-1).contiguous()
        self.dip_in = torch.empty_like(self.dip_target)
        self.dip_steps = []

    # -----------------------------------------------------------------------------------------
    def sparse_coding(self, stream=None, want_coefs=False):
        """Yb = blocks of X + L1/mu1; Phi = D * ISTA-PnP(Yb) for every block."""
        ops.im2col(self.X, self.L1, self.mu1_32, self.cfg.bb, self.rows_d, self.cols_d, self.n_pad, Yb=self.Yb,
                   stream=stream)
        return self._ista(self.cfg.Nit, stream, want_coefs=want_coefs)

    def _ista(self, Nit, stream, want_coefs=False, coefs=None, warm_start=False, max_workgroups=0):
        """All blocks' ISTA into self.phi: the per-pattern Gram path when planned, else lrs_ista_f32."""
        if self.pat_plan is not None:
            return ops.ista_pat(self.Yb, self.obs_pat, self.pat_plan, self.pat_ntiles, self.K, self.n, self.alpha,
                                self.thr, Nit, self.ista_ws, self.prox, phi=self.phi, coefs=coefs,
                                want_coefs=want_coefs, stream=stream, max_workgroups=max_workgroups,
                                warm_start=warm_start)
        return ops.ista(self.Yb, self.obs, self.D, self.n, self.alpha, self.thr, Nit, self.prox, phi=self.phi,
                        coefs=coefs, want_coefs=want_coefs, ws=self.ista_ws, stream=stream,
                        max_workgroups=max_workgroups, warm_start=warm_start)

    def sparse_coding_range(self, b0: int, b1: int, stream=None):
        """Phi rows [b0, b1) only (the blocks of one task-parallel worker, lrspnp.dist.DipTaskSplit)."""
        if b1 <= b0:
            return
        ops.im2col(self.X, self.L1, self.mu1_32, self.cfg.bb, self.rows_d[b0:b1], self.cols_d[b0:b1], self.n_pad,
                   Yb=self.Yb[b0:b1], stream=stream)
        ws = self.ista_ws
        if self.pat_plan is not None:   # a block range runs the row-split kernel, on a workspace of its own
            if getattr(self, "_rs_ws", None) is None:
                self._rs_ws = ops.ista_workspace(self.n, self.K, self.prox, self.Yb.device)
            ws = self._rs_ws
        ops.ista(self.Yb[b0:b1], self.obs[b0:b1], self.D, self.n, self.alpha[b0:b1], self.thr[b0:b1], self.cfg.Nit,
                 self.prox, phi=self.phi[b0:b1], ws=ws, stream=stream)

    def admm(self, stream=None):
        """col2im + closed-form X + dual updates from the current Phi and U (main_LRS_PnP.py:324-366)."""
        ops.admm_update(self.X, self.L1, self.L2, self.Y, self.M, self.U, self.phi, self.cfg.bb, self.grid,
                        self.gamma32, self.mu1_32, self.mu2_32, norms=self.norms,
                        stream=stream or torch.cuda.current_stream())
        self.iteration += 1

    def low_rank(self, stream=None, s_out=None):
        warm = self.cfg.svt_warm and self.iteration > 0
        return ops.svt(self.X, self.L2, self.c2, self.tau, self.svt_ws, U=self.U, s_out=s_out, warm=warm,
                       stream=stream, method=self.cfg.svt_method)

    def low_rank_dip(self, stream):
        """U = DIP(X + L2/mu2) (…1-LiP.py:399-411) on `stream`; the host polls early stopping."""
        ops.unfolded_to_image(self.X, self.L2, self.c2, self.H, self.W, self.dip_in, stream=stream)
        with torch.cuda.stream(stream):
            img = self.dip.run(self.dip_target, self.dip_in, self.dip_mask, seed=self.cfg.dip_seed + self.iteration,
                               early_stop=self.dip.cfg.early_stop)
            ops.image_to_unfolded(img, self.H, self.W, self.U, stream=stream)
        self.dip_steps.append((self.dip.last_steps, self.dip.last_stop_epoch))

    def step(self):
        """One outer ADMM iteration (main_LRS_PnP.py:250-366), stream-ordered.  No host sync in
        the SVT mode; the DIP mode polls its early-stopping flag on the low-rank stream only."""
        if self.cfg.lowrank == "dip":
            if self.dip is None:
                raise LrsError("this LrsPnP was built without a DIP engine (dip_engine=False)")
            return self._step_dip()
        main = torch.cuda.current_stream()
        lr = self.lowrank_stream
        warm = self.cfg.svt_warm and self.iteration > 0
        stream_wait(lr, main)
        # low-rank prox, first half (whole chip, ~0.2 ms): fp64 Gram (+ Jacobi warm-start products)
        ops.svt_gram(self.X, self.L2, self.c2, self.svt_ws, warm=warm, stream=lr, method=self.cfg.svt_method)
        if self.comm is not None:
            self.comm.allreduce_(self.gram, lr)       # the cube's Gram = sum of the slabs' Grams
        gram_done = lr.record_event()
        # second half: the one-workgroup eigensolver then runs beside the sparse coding
        mw = self.cfg.svt_multi_wg
        if mw not in ("auto", "on", "off"):
            raise LrsError(f"unknown svt_multi_wg {mw!r} (auto | on | off)")
        ops.svt_finish(self.X, self.L2, self.c2, self.tau, self.svt_ws, self.U, warm=warm, stream=lr,
                       method=self.cfg.svt_method, multi_wg=mw == "on" or (mw == "auto" and self.comm is not None))
        ops.im2col(self.X, self.L1, self.mu1_32, self.cfg.bb, self.rows_d, self.cols_d, self.n_pad, Yb=self.Yb,
                   stream=main)
        if self.cfg.svt_gram_first or self.cfg.svt_method == "jacobi":
            # the Gram gets the chip before the sparse-coding kernel fills it, so the ~7 ms Jacobi
            # solve starts at once; the tridiagonal chain fits inside the sparse coding even when
            # its Gram waits for the first sparse-coding workgroups to retire
            main.wait_event(gram_done)
        self._ista(self.cfg.Nit, main)
        stream_wait(main, lr)
        ops.admm_update(self.X, self.L1, self.L2, self.Y, self.M, self.U, self.phi, self.cfg.bb, self.grid,
                        self.gamma32, self.mu1_32, self.mu2_32, norms=self.norms, stream=main)
        self.iteration += 1

    def _step_dip(self):
        main = torch.cuda.current_stream()
        lr = self.lowrank_stream
        stream_wait(lr, main)
        # sparse coding is enqueued first so it runs beside the DIP training
        ops.im2col(self.X, self.L1, self.mu1_32, self.cfg.bb, self.rows_d, self.cols_d, self.n_pad, Yb=self.Yb,
                   stream=main)
        rs = self.n_pad > 64 and self.D.shape[1] <= 512   # the row-split kernel (warm start) serves
        sl = max(1, min(int(self.cfg.ista_slices_dip), self.cfg.Nit)) if rs else 1
        if sl == 1:
            self._ista(self.cfg.Nit, main, max_workgroups=self.cfg.ista_max_wg_dip)
        else:   # time-sliced: Nit split over `sl` launches continuing from the coefficients
            if getattr(self, "_coefs", None) is None:
                self._coefs = torch.empty((self.nb, self.D.shape[1]), dtype=torch.float32, device=self.Yb.device)
            done = 0
            for k in range(sl):
                it = (self.cfg.Nit * (k + 1)) // sl - done
                self._ista(it, main, coefs=self._coefs, want_coefs=True, warm_start=k > 0,
                           max_workgroups=self.cfg.ista_max_wg_dip)
                done += it
        if self.cfg.ista_dip_order == "before":
            stream_wait(lr, main)
        elif self.cfg.ista_dip_order != "beside":
            raise LrsError(f"unknown ista_dip_order {self.cfg.ista_dip_order!r} (beside | before)")
        self.low_rank_dip(lr)
        stream_wait(main, lr)
        ops.admm_update(self.X, self.L1, self.L2, self.Y, self.M, self.U, self.phi, self.cfg.bb, self.grid,
                        self.gamma32, self.mu1_32, self.mu2_32, norms=self.norms, stream=main)
        self.iteration += 1

    def convergence(self):
        """state_convergence (main_LRS_PnP.py:23-25) of X, lambda_1, lambda_2 for the last step."""
        norms = self.norms
        if self.comm is not None:
            norms = norms.clone()
            self.comm.allreduce_(norms, torch.cuda.current_stream())
        return torch.log(torch.sqrt(norms)).cpu().tolist()
