"""Pinned-buffer placement vs PCIe copy rate: allocate pinned buffers with this thread bound to the CPUs of NUMA node
0 and then node 1 (first touch / allocation on that node), time a 512 MiB D2H, a 512 MiB H2D and both at once on two
streams, and print the GPU's own NUMA node (from its PCI bus id)."""
import os
import time

import torch


def cpus_of(node):
    out = set()
    for part in open("/sys/devices/system/node/node%d/cpulist" % node).read().strip().split(","):
        a, _, b = part.partition("-")
        out.update(range(int(a), int(b or a) + 1))
    return out


def numa_of(ptr, size):
    nodes = {}
    for line in open("/proc/self/numa_maps"):
        parts = line.split()
        start = int(parts[0], 16)
        if ptr <= start < ptr + size:
            for p in parts[1:]:
                if p.startswith("N") and "=" in p:
                    k, v = p.split("=")
                    nodes[k] = nodes.get(k, 0) + int(v)
    return nodes


props = torch.cuda.get_device_properties(0)
bus = "%04x:%02x:%02x.0" % (getattr(props, "pci_domain_id", 0), props.pci_bus_id, props.pci_device_id)
try:
    gnode = open("/sys/bus/pci/devices/%s/numa_node" % bus).read().strip()
except OSError as ex:
    gnode = repr(ex)
print("gpu pci", bus, "numa_node", gnode, flush=True)
dev = torch.device("cuda", 0)
nw = 64 << 20
d = torch.zeros(nw, dtype=torch.int64, device=dev)
d2 = torch.zeros(nw, dtype=torch.int64, device=dev)
sa, sb = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
aff = os.sched_getaffinity(0)
keep = []
for node in (0, 1, 0, 1):
    cpus = cpus_of(node) & aff
    os.sched_setaffinity(0, cpus)
    h = torch.empty((1120 << 20) // 8 + 2, dtype=torch.int64, pin_memory=True)
    hin = torch.empty(nw, dtype=torch.int64, pin_memory=True)
    os.sched_setaffinity(0, aff)
    keep += [h, hin]

    def t(fn, k=3):
        r = []
        for _ in range(k):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            r.append("%.2f" % ((time.perf_counter() - t0) * 1e3))
        return r

    def both():
        with torch.cuda.stream(sa):
            d2.copy_(hin, non_blocking=True)
        with torch.cuda.stream(sb):
            h[:nw].copy_(d, non_blocking=True)

    print("alloc on node %d: out %s in %s | d2h %s h2d %s both %s" % (
        node, numa_of(h.data_ptr(), h.numel() * 8), numa_of(hin.data_ptr(), hin.numel() * 8),
        t(lambda: h[:nw].copy_(d, non_blocking=True)), t(lambda: d2.copy_(hin, non_blocking=True)), t(both)),
        flush=True)
