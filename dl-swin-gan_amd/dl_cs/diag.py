"""Diagnostic switches.

The engines keep a few superseded kernels reachable for A/B measurement (the
f32-MFMA convolutions, the bf16 3-plane patch GEMMs, the in-register thin-end
split, ...) and the tests compare them with the default dispatch.  Their
environment variables are read only when ``DLCS_DIAG=1`` is set as well, so a
production process runs the default dispatch whatever else its environment
holds.  The native library's switches exist only in its DIAG build
(``make -C dl-swin-gan_amd/csrc DIAG=1`` -> ``libdlcs_hip_diag.so``, selected with
``DLCS_HIP_LIB``; ``dlcs_knob`` in ``csrc/dlcs_common.h``), which also carries the
superseded bf16 3-plane conv and NT GEMM that ``DLCS_EMBED_X6`` reaches.
"""
import os


def enabled() -> bool:
    return os.environ.get("DLCS_DIAG", "0") == "1"


def knob(name: str, default: str) -> str:
    """``os.environ[name]`` under ``DLCS_DIAG=1``, else ``default``."""
    return os.environ.get(name, default) if enabled() else default
