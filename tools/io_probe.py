"""Page-cache file I/O rates (tool, not product): pwrite / pread of a 1 GiB file in 32 MiB
chunks from 1, 2, 4 and 8 threads -- is the CSV file path's single-threaded I/O loop the
bound?  Prints one JSON object.  usage: python tools/io_probe.py [DIR]"""
import json
import os
import sys
import threading
import time

import numpy as np

d = sys.argv[1] if len(sys.argv) > 1 else "/tmp"
path = os.path.join(d, "rss_io_probe.bin")
total, chunk = 1 << 30, 32 << 20
buf = np.random.default_rng(0).integers(0, 255, chunk, dtype=np.uint8)
mv = memoryview(buf)
res = {"dir": d, "bytes": total, "chunk": chunk}


def run(threads, op):
    fd = os.open(path, os.O_RDWR | os.O_CREAT | (os.O_TRUNC if op == "write" else 0), 0o644)
    n = total // chunk
    bufs = [bytearray(chunk) for _ in range(threads)]

    def work(t):
        for k in range(t, n, threads):
            if op == "write":
                os.pwrite(fd, mv, k * chunk)
            else:
                os.preadv(fd, [bufs[t]], k * chunk)
    t0 = time.perf_counter()
    ths = [threading.Thread(target=work, args=(t,)) for t in range(threads)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    dt = time.perf_counter() - t0
    os.close(fd)
    return total / dt / 1e9


for threads in (1, 2, 4, 8):
    w = [run(threads, "write") for _ in range(2)]
    r = [run(threads, "read") for _ in range(2)]
    res["threads_%d" % threads] = {"write_GBs": max(w), "read_GBs": max(r)}
os.unlink(path)
print(json.dumps(res))
