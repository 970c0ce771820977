"""dl_cs on MI355X: the Swin-unrolled cine reconstruction hot path of
tjtiger86/dl-swin-gan (dl_cs.models / dl_cs.mri API), running hand-written
HIP/CDNA4 kernels (libdlcs_hip.so) through a thin C-ABI."""
__version__ = "0.1.0"
