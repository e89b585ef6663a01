"""Does a CU-masked HIP stream (hipExtStreamCreateWithCUMask) partition the chip, and do torch
work and captured graphs run on it?  Times a fixed fp32 matmul chain on: the default stream; one
stream masked to 64 CUs; four 64-CU streams concurrently; four unmasked streams concurrently."""
import ctypes as C
import time

import torch

hip = C.CDLL("libamdhip64.so")
hip.hipExtStreamCreateWithCUMask.argtypes = [C.POINTER(C.c_void_p), C.c_uint32, C.POINTER(C.c_uint32)]


def masked_stream(bits):
    n = 8   # 256 CUs
    arr = (C.c_uint32 * n)()
    for b in bits:
        arr[b // 32] |= 1 << (b % 32)
    s = C.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(C.byref(s), n, arr)
    assert rc == 0, rc
    return torch.cuda.ExternalStream(s.value)


def work(a, b, reps):
    for _ in range(reps):
        c = a @ b
    return c


def timeit(fn):
    torch.cuda.synchronize()
    t = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) * 1e3


def main():
    dev = torch.device("cuda")
    print("CUs", torch.cuda.get_device_properties(0).multi_processor_count)
    a = torch.randn(4096, 4096, device=dev)
    b = torch.randn(4096, 4096, device=dev)
    R = 20
    work(a, b, 2)
    print("default stream      %.2f ms" % timeit(lambda: work(a, b, R)))
    for name, parts in [("contiguous", [list(range(64 * e, 64 * e + 64)) for e in range(4)]),
                        ("interleaved", [list(range(e, 256, 4)) for e in range(4)])]:
        ss = [masked_stream(p) for p in parts]
        def one():
            with torch.cuda.stream(ss[0]):
                work(a, b, R)
        print(f"{name}: one 64-CU stream  %.2f ms" % timeit(one))
        def four():
            for s in ss:
                with torch.cuda.stream(s):
                    work(a, b, R)
        print(f"{name}: four 64-CU streams %.2f ms (4x the work)" % timeit(four))
    us = [torch.cuda.Stream() for _ in range(4)]
    def four_u():
        for s in us:
            with torch.cuda.stream(s):
                work(a, b, R)
    print("four unmasked streams %.2f ms (4x the work)" % timeit(four_u))
    # graph capture on a masked stream, replayed there
    s = masked_stream(range(64))
    g = torch.cuda.CUDAGraph()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        work(a, b, 1)
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s):
            c = work(a, b, R)
    ref = a @ b
    def rep():
        with torch.cuda.stream(s):
            g.replay()
    print("graph on 64-CU stream %.2f ms" % timeit(rep))
    print("graph result ok", torch.allclose(c, ref))


if __name__ == "__main__":
    main()
