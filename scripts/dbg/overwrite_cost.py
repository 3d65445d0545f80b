"""What replacing an existing 250-MB file costs the writer: open(O_TRUNC) +
write, against rename-away + the same write with the old file unlinked on
another thread, against writing a new file (the page cache warm, the same
bytes each time)."""
import os
import tempfile
import threading
import time

d = tempfile.mkdtemp()
path = os.path.join(d, "x.ply")
buf = os.urandom(1 << 20) * 250


def write(p):
    fd = os.open(p, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
    mv = memoryview(buf)
    off = 0
    while off < len(buf):
        off += os.write(fd, mv[off:off + (32 << 20)])
    os.close(fd)


for rep in range(3):
    if os.path.exists(path):
        os.unlink(path)
    t0 = time.perf_counter(); write(path); t1 = time.perf_counter()
    t2 = time.perf_counter(); write(path); t3 = time.perf_counter()  # overwrite (truncate)
    t4 = time.perf_counter()
    old = path + ".old"
    os.rename(path, old)
    th = threading.Thread(target=os.unlink, args=(old,))
    th.start()
    write(path)
    t5 = time.perf_counter()
    th.join()
    t6 = time.perf_counter()
    print(f"new {1e3 * (t1 - t0):.1f} ms, overwrite {1e3 * (t3 - t2):.1f} ms, "
          f"rename + background unlink {1e3 * (t5 - t4):.1f} ms (unlink done {1e3 * (t6 - t4):.1f})", flush=True)
os.unlink(path)
os.rmdir(d)
