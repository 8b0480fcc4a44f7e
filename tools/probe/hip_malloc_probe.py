import ctypes, time, torch
torch.cuda.init(); torch.zeros(1, device="cuda")
import glob, os; hip = ctypes.CDLL(glob.glob(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so*"))[0])
for mb in (40, 80, 320, 1024, 40, 320):
    p = ctypes.c_void_p()
    torch.cuda.synchronize()
    t0 = time.perf_counter(); rc = hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(mb << 20)); t1 = time.perf_counter()
    hip.hipMemset(p, 0, ctypes.c_size_t(mb << 20)); hip.hipDeviceSynchronize(); t2 = time.perf_counter()
    hip.hipFree(p); t3 = time.perf_counter()
    print(f"{mb} MB: malloc {(t1-t0)*1e3:.3f} ms, first memset {(t2-t1)*1e3:.3f} ms, free {(t3-t2)*1e3:.3f} ms", flush=True)
