"""LIBSVM input straight to device CSR: host mirror of
org.apache.spark.mllib.util.MLUtils.loadLibSVMFile (mllib/util/MLUtils.scala:
62-151).  The parse runs in libcyclone (csrc/libsvm.cpp: parallel over line
ranges, native), and the CSR arrays go to HBM in one upload -- the resident
layout every sparse kernel here reads (labels, rowptr int64, colidx int32,
values fp64; unit weights)."""
from __future__ import annotations

import ctypes
import os

import numpy as np

from . import _native as N


def _threads(nthreads):
    if nthreads:
        return int(nthreads)
    return max(1, min(os.cpu_count() or 1, 16))


class _Parsed:
    def __init__(self, h):
        self._lib = N.load()
        self.handle = h
        n, nnz, nf = ctypes.c_int64(0), ctypes.c_int64(0), ctypes.c_int32(0)
        N.check(self._lib.cyc_libsvm_sizes(h, ctypes.byref(n), ctypes.byref(nnz),
                                           ctypes.byref(nf)))
        self.n, self.nnz, self.numFeatures = n.value, nnz.value, nf.value

    def host(self):
        labels = np.empty(self.n)
        rowptr = np.empty(self.n + 1, dtype=np.int64)
        colidx = np.empty(self.nnz, dtype=np.int32)
        values = np.empty(self.nnz)
        p = lambda a: a.ctypes.data_as(ctypes.c_void_p)
        N.check(self._lib.cyc_libsvm_copy(self.handle, p(labels), p(rowptr), p(colidx),
                                          p(values)))
        return labels, (rowptr, colidx, values), self.numFeatures

    def device(self, device="cuda", stream=None):
        import torch
        dev = torch.device(device)
        labels = torch.empty(self.n, dtype=torch.float64, device=dev)
        rowptr = torch.empty(self.n + 1, dtype=torch.int64, device=dev)
        colidx = torch.empty(max(self.nnz, 1), dtype=torch.int32, device=dev)[:self.nnz]
        values = torch.empty(max(self.nnz, 1), dtype=torch.float64, device=dev)[:self.nnz]
        N.check(self._lib.cyc_libsvm_upload(self.handle, N.ptr(labels), N.ptr(rowptr),
                                            N.ptr(colidx), N.ptr(values),
                                            N.stream_handle(stream)))
        return labels, (rowptr, colidx, values), self.numFeatures

    def __del__(self):
        try:
            if self.handle:
                self._lib.cyc_libsvm_destroy(self.handle)
                self.handle = None
        except Exception:
            pass


def _parse_text(text, numFeatures=-1, nthreads=None):
    if isinstance(text, str):
        text = text.encode()
    h = ctypes.c_void_p()
    N.check(N.load().cyc_libsvm_parse(text, len(text), int(numFeatures), _threads(nthreads),
                                      ctypes.byref(h)))
    return _Parsed(h)


def _parse_file(path, numFeatures=-1, nthreads=None):
    h = ctypes.c_void_p()
    N.check(N.load().cyc_libsvm_load_file(os.fsencode(path), int(numFeatures),
                                          _threads(nthreads), ctypes.byref(h)))
    return _Parsed(h)


def parseLibSVM(text, numFeatures=-1, nthreads=None):
    """parseLibSVMFile + computeNumFeatures over in-memory text: host arrays
    (labels, (rowptr, colidx, values), numFeatures)."""
    return _parse_text(text, numFeatures, nthreads).host()


def parseLibSVMFile(path, numFeatures=-1, nthreads=None):
    """Host arrays of a LIBSVM file (labels, (rowptr, colidx, values), numFeatures)."""
    return _parse_file(path, numFeatures, nthreads).host()


def loadLibSVMFile(path, numFeatures=-1, device="cuda", stream=None, nthreads=None):
    """MLUtils.loadLibSVMFile(sc, path, numFeatures) as one device-resident
    CSR block (DeviceInstanceBlock, unit weights): the rows of the file in
    order, labels and values bit-identical to the JVM parse."""
    from .optim import DeviceInstanceBlock
    labels, (rp, ci, v), nf = _parse_file(path, numFeatures, nthreads).device(device, stream)
    return DeviceInstanceBlock(labels, None, rowptr=rp, colidx=ci, values=v, numFeatures=nf)
