"""Diagnosis only (VERDICT r5 "what's weak" #1): the round-5 lifecycle of a
captured memset -- hipMemsetAsync on the capturing stream inside
torch.cuda.graph (which destroys the hipGraph_t after instantiating it), then
replays with Python work in between -- on a buffer the graph first fills with
0xff bytes.  Prints, per replay, the non-zero words left after the memset.
Companion of scripts/dbg/graph_memset.hip (the same question without torch).

    python scripts/dbg/graph_memset_torch.py [replays]
"""
import ctypes
import json
import sys

import torch

WORDS = 2176  # one view's histogram replicas in the library (8704 B)


def main():
    replays = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemsetAsync.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    bad = 0
    for keep in (False, True):
        h = torch.zeros(WORDS, dtype=torch.int32, device=dev)
        res = torch.zeros(2, dtype=torch.int64, device=dev)
        s = torch.cuda.Stream(dev)
        g = torch.cuda.CUDAGraph(keep_graph=keep)
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
            h.fill_(-1)
            rc = hip.hipMemsetAsync(ctypes.c_void_p(h.data_ptr()), 0, 4 * WORDS, ctypes.c_void_p(s.cuda_stream))
            res[0] = (h != 0).sum()
            res[1] = h[0]
        if keep:
            g.instantiate()
        for r in range(replays):
            junk = [bytearray(b"\xa5" * (8 + (i * 7919) % 505)) for i in range(3000)]  # host heap churn
            del junk
            with torch.cuda.stream(s):
                g.replay()
            torch.cuda.synchronize()
            nz, first = (int(x) for x in res.cpu())
            bad += nz != 0
            print(json.dumps({"variant": "torch_graph_keep" if keep else "torch_graph_destroyed", "replay": r,
                              "capture_rc": rc, "nonzero_words": nz, "word0": f"0x{first & 0xffffffff:08x}",
                              # the garbage against the device addresses the graph's nodes hold
                              "h_ptr": f"0x{h.data_ptr():x}", "res_ptr": f"0x{res.data_ptr():x}",
                              "ok": nz == 0}), flush=True)
        del g
    print(json.dumps({"torch": torch.__version__, "hip": torch.version.hip, "bad_replays": bad}), flush=True)


if __name__ == "__main__":
    main()
