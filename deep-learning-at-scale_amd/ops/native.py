"""Loader for the in-tree HIP kernel library ``wellflow/_C.so``.

There is no fallback: GPU code paths call :func:`lib` and get an ImportError with the
build instruction when the extension is missing (the CPU oracle paths never touch it).
"""
from __future__ import annotations

import importlib
import os

_LIB = None


def lib():
    """Return the loaded ``wellflow._C`` module (raises if it was not built)."""
    global _LIB
    if _LIB is None:
        import torch  # noqa: F401  (loads libtorch / libamdhip64 first)

        try:
            _LIB = importlib.import_module("wellflow._C")
        except ImportError as e:  # pragma: no cover - depends on the build
            here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
            raise ImportError(
                f"wellflow native extension not built ({e}). Run `python -m wellflow._build` "
                f"(expects {os.path.join(here, '_C.so')})."
            ) from e
    return _LIB


def available() -> bool:
    try:
        lib()
        return True
    except ImportError:
        return False


def gemm(A, B, M, N, K, *, a_mn=False, lda=None, b_mn=False, ldb=None, outF=None, outH=None,
         ldo=None, bias=None, mask=None, ldm=None, mask_scale=1.0, colsum=None, alpha=1.0,
         beta=0.0, act=0, atomic=False, ksplit=1, drop_p=0.0, seed=0, tile=0, seed_dev=None):
    """out = act(alpha * A(M,K) B(N,K)^T + beta*out + bias) (* mask), on MFMA.

    ``a_mn``/``b_mn`` select the MN-contiguous layout (X(r,k) = p[k*ld + r]).
    ``tile`` (MN x MN split-K atomic only): 1 = 256x128 8-wave tile, 2 = 128x288, 3 = 256x192.
    ``seed_dev`` (int64 GPU tensor): a device step counter mixed into the dropout seed.
    """
    if lda is None:
        lda = M if a_mn else K
    if ldb is None:
        ldb = N if b_mn else K
    if ldo is None:
        ldo = N
    if ldm is None:
        ldm = ldo
    lib().gemm(A, bool(a_mn), int(lda), B, bool(b_mn), int(ldb), int(M), int(N), int(K),
               int(ksplit), outF, outH, int(ldo), bias, mask, int(ldm), float(mask_scale), colsum,
               float(alpha), float(beta), int(act), bool(atomic), float(drop_p), int(seed), int(tile), seed_dev)
