"""Host page size vs PCIe copy rate (the C5 host-path slow state): anonymous 2 MiB-aligned
mappings advised MADV_NOHUGEPAGE (4 KiB pages) or MADV_HUGEPAGE (THP), touched, registered with hipHostRegister,
then a 512 MiB D2H, H2D and both at once. Also prints THP / IOMMU settings and the page size torch's pinned buffers
got (smaps)."""
import ctypes as C
import glob
import mmap
import time

import torch


def rd(p):
    try:
        return open(p).read().strip()
    except OSError as ex:
        return repr(ex)


print("thp enabled:", rd("/sys/kernel/mm/transparent_hugepage/enabled"), "defrag:",
      rd("/sys/kernel/mm/transparent_hugepage/defrag"), flush=True)
print("iommu groups:", len(glob.glob("/sys/kernel/iommu_groups/*")), "iommu dev:", glob.glob("/sys/class/iommu/*")[:4],
      "cmdline:", rd("/proc/cmdline")[:300], flush=True)


def smaps_of(ptr):
    out, cur = {}, False
    for line in open("/proc/self/smaps"):
        if "-" in line.split()[0] and not line.startswith(("Size", "Rss")):
            a, b = line.split()[0].split("-")
            cur = int(a, 16) <= ptr < int(b, 16)
            continue
        if cur and line.split()[0] in ("Size:", "Rss:", "AnonHugePages:", "KernelPageSize:", "Locked:"):
            out[line.split()[0][:-1]] = " ".join(line.split()[1:])
    return out


hip = C.CDLL("libamdhip64.so")
libc = C.CDLL("libc.so.6", use_errno=True)
libc.madvise.argtypes = [C.c_void_p, C.c_size_t, C.c_int]
MADV_HUGEPAGE, MADV_NOHUGEPAGE = 14, 15
dev = torch.device("cuda", 0)
nw = 64 << 20
nbytes = nw * 8
d = torch.zeros(nw, dtype=torch.int64, device=dev)
d2 = torch.zeros(nw, dtype=torch.int64, device=dev)
sa, sb = torch.cuda.Stream(dev), torch.cuda.Stream(dev)


def t(fn, k=4):
    r = []
    for _ in range(k):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        r.append("%.2f" % ((time.perf_counter() - t0) * 1e3))
    return r


keep = []


def registered(advice):
    size = nbytes + (2 << 20)
    m = mmap.mmap(-1, size, flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)
    base = C.addressof(C.c_char.from_buffer(m))
    al = (base + (2 << 20) - 1) & ~((2 << 20) - 1)
    libc.madvise(C.c_void_p(al), C.c_size_t(nbytes), advice)
    C.memset(C.c_void_p(al), 1, nbytes)  # touch
    rc = hip.hipHostRegister(C.c_void_p(al), C.c_size_t(nbytes), 0)
    arr = (C.c_int64 * nw).from_address(al)
    ten = torch.frombuffer(arr, dtype=torch.int64)
    keep.append((m, arr, ten))
    return ten, rc, al


tp = torch.empty((1120 << 20) // 8 + 2, dtype=torch.int64, pin_memory=True)
print("torch pinned:", smaps_of(tp.data_ptr()), "d2h", t(lambda: tp[:nw].copy_(d, non_blocking=True)), flush=True)
for name, adv in (("4K pages", MADV_NOHUGEPAGE), ("THP", MADV_HUGEPAGE), ("4K pages", MADV_NOHUGEPAGE),
                  ("THP", MADV_HUGEPAGE)):
    ho, rc1, a1 = registered(adv)
    hi, rc2, a2 = registered(adv)

    def both():
        with torch.cuda.stream(sa):
            d2.copy_(hi, non_blocking=True)
        with torch.cuda.stream(sb):
            ho.copy_(d, non_blocking=True)

    print("%-8s reg rc %d/%d %s | d2h %s h2d %s both %s" % (
        name, rc1, rc2, smaps_of(a1), t(lambda: ho.copy_(d, non_blocking=True)),
        t(lambda: d2.copy_(hi, non_blocking=True)), t(both)), flush=True)
