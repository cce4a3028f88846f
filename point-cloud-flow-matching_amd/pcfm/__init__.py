"""pcfm: MI355X-native hot path of Point-Cloud-Flow-Matching.

Layout of this directory (put it on sys.path; the reference does the same with
third_party/pvcnn, models.py:9-13):

  csrc/        HIP kernels for gfx950 + the C ABI of include/pcfm.h
  pcfm/        host side: ctypes binding (_lib), tensor ops with the
               reference's native-module signatures (ops), flow models,
               train step, samplers
  modules/     drop-in for the reference's `modules` package (PVCNN)
  chamfer3D/   drop-in for ChamferDistancePytorch/chamfer3D/dist_chamfer_3D.py
  PyTorchEMD/  drop-in for PyTorchEMD/emd.py
"""
__all__ = ["ops"]
