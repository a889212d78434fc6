"""PerfPolicy: the typed switchboard of every hot-path kernel / fusion choice.

The models consult ``policy()`` when they run (not at import), so a policy can be changed for a
scope (``use_policy``) inside one process -- the fused-vs-library convergence A/B runs both
paths side by side -- and it is recorded with every benchmark line and checkpoint
(``to_dict``). Defaults are the measured-best settings (each field names its evidence); the
``CML_*`` environment variables of round 2 still override a default when set, so older run
scripts keep working, but the effective policy is what gets recorded.

``PerfPolicy.library()`` is the reference configuration with every own kernel and fusion off:
MIOpen / hipBLASLt convolutions and GEMMs and PyTorch's BatchNorm composition.
"""
from __future__ import annotations

import contextlib
import dataclasses
import os
from dataclasses import dataclass, fields
from typing import Any, Dict, Iterator


def _env_bool(name: str, default: bool) -> bool:
    v = os.environ.get(name)
    return default if v is None else v == "1"


def _env_int(name: str, default: int) -> int:
    v = os.environ.get(name)
    return default if v is None else int(v)


def _env_str(name: str, default: str) -> str:
    return os.environ.get(name, default)


@dataclass
class PerfPolicy:
    # ---------------------------------------------------------------- BatchNorm
    fused_bn: bool = True                 # bn_act.hip BN (+residual) (+ReLU); False: PyTorch BN
    residual_link: bool = True            # residual gradients absorbed by GEMM epilogues
    # ---------------------------------------------------------------- ResNet stem / head
    fuse_stem_conv: bool = True           # stem_conv.hip conv + BN stats, one-pass weight grad
    fuse_stem_pool: bool = True           # BN + ReLU + max-pool in one pass
    pool_link: bool = True                # pool backward sums layer1.0's downsample gradient
    stem_pool_gather: bool = True         # stem wgrad gathers the pool input gradient itself
    stem_pad4: bool = True                # 3 -> 4 input channels for MIOpen's NHWC kernels
    nhwc_avgpool: bool = True             # global average pool with an NHWC backward
    # ---------------------------------------------------------------- 1x1 convolutions
    conv1x1_gemm: str = "auto"            # auto | gemm | miopen (library fwd / dgrad choice)
    fused_conv1x1: bool = True            # conv1x1 + BN statistics / bn2 prologue kernels
    conv1x1g: str = "auto"                # fused-kernel family: auto | quad | regstage
    own_wgrad1x1: bool = True             # wgrad1x1.hip for the OWN_WGRAD_SHAPES set
    wgrad1x1_set: str = "wide"            # core (5 shapes) | all (9) | wide (all + downsample)
    fused_bn3_bwd: bool = True            # identity-tail backward inside conv3's kernels
    fused_bn3_bwd_max_planes: int = 128
    recompute_tail: bool = True           # identity tails without a stored z3
    recompute_tail_max_planes: int = 256
    recompute_down_tail: bool = True      # stride-1 downsample tail without z3 / zd
    recompute_down_tail_s2: bool = True   # stride-2 downsample tails on the recompute kernels
    down_tail_s2_max_cin: int = 512
    fuse_down_bn: bool = True             # relu(bn3(z) + bn_d(zd)) as one op
    gram_stats: bool = True               # recompute-tail BN statistics from the Gram matrix
    cat_bnsums: bool = True               # bn2's backward sums in the cat GEMM's epilogue
    cat_bnsums_maxc: int = 256
    s2_link_dgrad: bool = True            # compact stride-2 gradient added in conv1's dgrad
    down_s2_compact: bool = True          # non-recompute stride-2 downsample (layer 4) as a
                                          # stride-1 GEMM of x[:, :, ::2, ::2], compact gradient
    bn_affine_kernel: bool = True         # one-launch BN affine (sc, bi)
    # ---------------------------------------------------------------- 3x3 convolutions
    own_dgrad3x3: bool = True             # conv_gemm.hip data gradient
    conv3x3_bn_stats: bool = True         # conv_gemm.hip forward + BN statistics epilogue
    bn1_dgrad_sums: bool = True           # bn1's backward sums in the 3x3 dgrad epilogue
    bn1_sums_lib_conv1: bool = False      # ... also behind a library conv1 (layers 3-4): 0.4-0.6
                                          # ms/step SLOWER (pass 26, profiles/r03_26/)
    own_wgrad3x3: bool = True             # wgrad3x3.hip weight gradient
    own_wgrad3x3_s2: bool = True          # stride-2 3x3 weight gradient on the wgrad DMA kernel
    wgrad3x3_s2_min_ci: int = 256         # ... for Ci >= this (the 128-channel layer-2 conv: MIOpen)
    own_wgrad1x1_s2: bool = True          # stride-2 1x1 (downsample) weight gradient on the same
                                          # kernel, one tap (was MIOpen)
    c1_dgrad64_gemm: bool = True          # layer 1.0 conv1 (64 -> 64) data gradient as a GEMM that
                                          # absorbs the downsample's dX (no pool two-gradient sum)
    own_conv3x3_s2: bool = True           # stride-2 3x3: conv_gemm forward + BN stats, parity-class
                                          # data gradient (+ bn1 backward sums)
    side_wgrad: bool = True               # 3x3 weight gradients on a side stream, concurrent with
                                          # the same conv's data-gradient / BN-backward kernels,
    side_wgrad_min_batch: int = 1024      # ... at per-GPU batches >= this: batch 2560 -0.2 to
                                          # -0.6 ms/step, batch 256 +0.3 ms (profiles/r06_53/)
    link_dgrad_plain: bool = True         # 1x1 data gradients that absorb a plain parked gradient
                                          # and would run on hipBLASLt (N 64): the fused 1x1 kernel
                                          # with the add in its epilogue (conv1x1_link, no mask)
    side_wgrad_1x1: bool = False          # ... also the 1x1 convs' weight gradients: batch 2560
                                          # 141.77 / 140.83 / 141.58 vs 141.15 / 140.73 / 141.84 ms
                                          # (noise level, profiles/r06_55/)
    fin_dgamma: bool = True               # BN parameter gradients from the backward sums' finalize
                                          # launch (no bn_bwd_coeffs launch: batch-256 tails)
    fin_affine: bool = True               # BN affine (gamma invstd, beta - mean sc) from the
                                          # statistics' finalize launch (no bn_affine launch)
    batch_wlayouts: bool = True           # all 3x3 weight layouts of a ResNet forward in one launch
    # ---------------------------------------------------------------- transformers / engine
    attn_kernel: bool = True              # MFMA attention for short sequences (BERT)
    flash_attn: bool = True               # flash_attn.hip for head-dim-128 (GQA, causal) attention
                                          # (Llama); False: SDPA (AOTriton kernels on ROCm torch)
    multi_copy: bool = True               # multi-tensor HIP copy for gradient capture
    batched_workers: bool = True          # virtual workers as one batched fwd/bwd (BERT)
    own_gemm: bool = True                 # gemm.hip for transformer linears with >= 128 tiles
    own_gemm128: bool = True              # ... and gemm128.hip (128 x 128 tiles) below that: the
                                          # BERT per-rank shapes (8192 x 768 outputs) run 1.15-1.8x
                                          # hipBLASLt (profiles/r05_05/gemm.jsonl)
    fused_ffn: bool = True                # BERT FFN on gemm.hip: bias + GELU in fc1's epilogue,
                                          # GELU backward + bias gradient in the dgrad epilogue
    padded_logits: bool = True            # biased linears with N % 8 != 0 (BERT MLM head) write
                                          # 16-B aligned padded rows; the CE backward emits the
                                          # bias gradient (no column-sum pass over R x V)
    own_gemm_conv1x1: bool = True         # ResNet 1x1 convs that run as plain GEMMs (layers 3-4
                                          # forward / data gradient) on gemm.hip, not hipBLASLt
    nt_wgrad: bool = True                 # bias-free (Llama) linears: weight gradient as an NT GEMM
                                          # on transposed operands (1.3-1.57 vs 0.9-1.15 PFLOP/s for
                                          # hipBLASLt's dY^T X layout, profiles/r05_06/llama_gemm.jsonl)
    own_linear_wgrad: bool = True         # transformer-linear weight gradients dY^T X on
                                          # wgrad1x1.hip (token rows as NHWC pixels), not hipBLASLt,
                                          # up to BERT-base sizes (N K <= 4 M)

    @classmethod
    def from_env(cls) -> "PerfPolicy":
        """Defaults, overridden by the round-2 ``CML_*`` variables where set."""
        return cls(
            fused_bn=_env_bool("CML_FUSED_BN", True),
            fuse_stem_conv=_env_bool("CML_FUSE_STEM_CONV", True),
            fuse_stem_pool=_env_bool("CML_FUSE_STEM_POOL", True),
            pool_link=_env_bool("CML_POOL_LINK", True),
            stem_pool_gather=_env_bool("CML_STEM_POOL_GATHER", True),
            stem_pad4=_env_bool("CML_STEM_PAD4", True),
            nhwc_avgpool=_env_bool("CML_NHWC_AVGPOOL", True),
            conv1x1_gemm=_env_str("CML_CONV1X1_GEMM", "auto"),
            fused_conv1x1=_env_bool("CML_FUSED_CONV1X1", True),
            conv1x1g={"0": "regstage", "3": "quad"}.get(os.environ.get("CML_C1G", ""), "auto"),
            own_wgrad1x1=_env_bool("CML_WGRAD1X1", True),
            wgrad1x1_set=_env_str("CML_WGRAD1X1_SET", "wide"),
            fused_bn3_bwd=_env_bool("CML_FUSED_BN3_BWD", True),
            fused_bn3_bwd_max_planes=_env_int("CML_FUSED_BN3_BWD_MAX_PLANES", 128),
            recompute_tail=_env_bool("CML_RECOMPUTE_TAIL", True),
            recompute_tail_max_planes=_env_int("CML_RECOMPUTE_TAIL_MAX_PLANES", 256),
            recompute_down_tail=_env_bool("CML_RECOMPUTE_DOWN_TAIL", True),
            recompute_down_tail_s2=_env_bool("CML_RECOMPUTE_DOWN_TAIL_S2", True),
            down_tail_s2_max_cin=_env_int("CML_DOWN_TAIL_S2_MAX_CIN", 512),
            fuse_down_bn=_env_bool("CML_FUSE_DOWN_BN", True),
            gram_stats=_env_bool("CML_GRAM_STATS", True),
            cat_bnsums=_env_bool("CML_CAT_BNSUMS", True),
            cat_bnsums_maxc=_env_int("CML_CAT_BNSUMS_MAXC", 256),
            s2_link_dgrad=_env_bool("CML_S2_LINK_DGRAD", True),
            down_s2_compact=_env_bool("CML_DOWN_S2_COMPACT", True),
            bn_affine_kernel=_env_bool("CML_BN_AFFINE_KERNEL", True),
            own_dgrad3x3=_env_bool("CML_DGRAD3X3", True),
            conv3x3_bn_stats=_env_bool("CML_CONV3X3_BN_STATS", True),
            bn1_dgrad_sums=_env_bool("CML_BN1_DGRAD_SUMS", True),
            bn1_sums_lib_conv1=_env_bool("CML_BN1_SUMS_LIB_CONV1", False),
            own_wgrad3x3=_env_bool("CML_WGRAD3X3", True),
            own_wgrad3x3_s2=_env_bool("CML_WGRAD3X3_S2", True),
            wgrad3x3_s2_min_ci=int(os.environ.get("CML_WGRAD3X3_S2_MIN_CI", "256")),
            own_wgrad1x1_s2=_env_bool("CML_WGRAD1X1_S2", True),
            c1_dgrad64_gemm=_env_bool("CML_C1_DGRAD64", True),
            own_conv3x3_s2=_env_bool("CML_CONV3X3_S2", True),
            side_wgrad=_env_bool("CML_SIDE_WGRAD", True),
            side_wgrad_min_batch=_env_int("CML_SIDE_WGRAD_MIN_BATCH", 1024),
            side_wgrad_1x1=_env_bool("CML_SIDE_WGRAD_1X1", False),
            link_dgrad_plain=_env_bool("CML_LINK_DGRAD_PLAIN", True),
            fin_dgamma=_env_bool("CML_FIN_DGAMMA", True),
            fin_affine=_env_bool("CML_FIN_AFFINE", True),
            batch_wlayouts=_env_bool("CML_BATCH_WLAYOUTS", True),
            attn_kernel=_env_bool("CML_ATTN_KERNEL", True),
            flash_attn=_env_bool("CML_FLASH_ATTN", True),
            multi_copy=_env_bool("CML_MULTI_COPY", True),
            batched_workers=_env_bool("CML_BATCHED_WORKERS", True),
            own_gemm=_env_bool("CML_OWN_GEMM", True),
            own_gemm128=_env_bool("CML_OWN_GEMM128", True),
            fused_ffn=_env_bool("CML_FUSED_FFN", True),
            own_gemm_conv1x1=_env_bool("CML_OWN_GEMM_CONV1X1", True),
            own_linear_wgrad=_env_bool("CML_OWN_LINEAR_WGRAD", True),
            nt_wgrad=_env_bool("CML_NT_WGRAD", True),
            padded_logits=_env_bool("CML_PADDED_LOGITS", True),
        )

    @classmethod
    def library(cls) -> "PerfPolicy":
        """Every own kernel and fusion off: MIOpen / hipBLASLt + PyTorch BatchNorm."""
        off: Dict[str, Any] = {}
        for f in fields(cls):
            if f.type in ("bool", bool):
                off[f.name] = False
        off.update(conv1x1_gemm="miopen", conv1x1g="regstage")
        return cls(**off)

    def replace(self, **kw) -> "PerfPolicy":
        return dataclasses.replace(self, **kw)

    def to_dict(self) -> Dict[str, Any]:
        return dataclasses.asdict(self)

    def validate(self) -> "PerfPolicy":
        if self.conv1x1_gemm not in ("auto", "gemm", "miopen"):
            raise ValueError(f"conv1x1_gemm must be auto | gemm | miopen, not {self.conv1x1_gemm!r}")
        if self.conv1x1g not in ("auto", "quad", "regstage"):
            raise ValueError(f"conv1x1g must be auto | quad | regstage, not "
                             f"{self.conv1x1g!r}")
        if self.wgrad1x1_set not in ("core", "all", "wide"):
            raise ValueError(f"wgrad1x1_set must be core | all | wide, not "
                             f"{self.wgrad1x1_set!r}")
        return self


_CURRENT = PerfPolicy.from_env().validate()
_NATIVE_SYNCED = None


def env_switches() -> Dict[str, str]:
    """The ``CML_*`` variables set in this process (the policy's overrides and the native
    launchers' A/B switches such as CML_CONV3P / CML_CONV_GEMM2, which the policy does not hold),
    recorded beside the policy in benchmark lines; the bench launcher's own are left out."""
    return {k: v for k, v in sorted(os.environ.items())
            if k.startswith("CML_") and not k.startswith("CML_BENCH_")}


def policy() -> PerfPolicy:
    """The policy in force (read by the models at call time)."""
    return _CURRENT


def _sync_native(p: PerfPolicy) -> None:
    """Push the native-side switches (kernel-family choice inside the C++ launchers)."""
    global _NATIVE_SYNCED
    mode = {"regstage": 0, "auto": 2, "quad": 3}[p.conv1x1g]
    if _NATIVE_SYNCED == mode:
        return
    try:
        from .ops.native import lib
        L = lib()
    except Exception:       # no extension (CPU-only environments): nothing to push
        return
    L.set_conv1x1g_mode(mode)
    _NATIVE_SYNCED = mode


def set_policy(p: PerfPolicy) -> PerfPolicy:
    """Install ``p`` process-wide; returns the previous policy."""
    global _CURRENT
    prev = _CURRENT
    _CURRENT = p.validate()
    if prev.conv1x1g != p.conv1x1g or _NATIVE_SYNCED is not None:
        _sync_native(p)
    return prev


def ensure_native_synced() -> None:
    """Called once the extension is loaded: apply the current policy's native switches."""
    _sync_native(_CURRENT)


@contextlib.contextmanager
def use_policy(p: PerfPolicy) -> Iterator[PerfPolicy]:
    prev = set_policy(p)
    try:
        yield p
    finally:
        set_policy(prev)
