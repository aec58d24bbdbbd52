"""adipose_amd — MI355X-native (gfx950) U-Net segmentation engine, a drop-in for the hot path of
MAGIC-SCAN/adipose_tissue-unet (Segmentation/train_adipose_unet_v3.py, segmentation_inference.py,
full_evaluation_enhanced.py). Compute runs only in libadipose_hip.so (hand-written HIP kernels
behind a C ABI, include/adipose_hip.h); PyTorch provides device memory, streams and RCCL."""

__version__ = "0.1.0"
