"""Process-level choices made before the library loads.

USE_TORCH: import PyTorch before libfrender_hip.so, so that the process holds one HIP runtime (torch's),
which torch.distributed (RCCL) needs to move buffers the library wrote.  The single-GPU command lines
(`python -m frender_amd scan|demux` without --gpus) touch no torch tensor and turn it off: the import
costs ~2 s of each command's start.  Multi-rank runs, bench.py and library users keep it on."""
USE_TORCH = True
