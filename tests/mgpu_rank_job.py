"""The RCCL rank-per-process form of wsg_mgpu_encode_gather at world > 1 on
one GPU (run by tests/test_gpu_c5.py::test_mgpu_rank_form_world_n in a
process of its own).

wsg_mgpu_create_rank loads RCCL through $WSG_RCCL_LIB; the test points it at
tests/cpp/_build/libloopback_rccl.so, a test double whose ranks are threads
of one process sharing the GPU (its header says what it keeps of NCCL's
semantics).  Every rank here is a thread holding its own wsg_mgpu handle,
exactly as a process would: its shard encoded by its own context, then the
status and chunk-size all-gathers and the grouped per-chunk Send/Recv into
the root — the code a real multi-process job runs.  The root's wire and
offsets are checked against the oracle's encode of the whole job.

Prints one JSON line: {"cases": [...], "loopback_errors": N}.
"""
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle  # noqa: E402
import cppserver_amd as ca  # noqa: E402
from cppserver_amd import shard  # noqa: E402
from cppserver_amd import workloads as wl  # noqa: E402


def ragged_job(n, seed):
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, 3000, n)
    big = rng.random(n) < 0.05
    lens[big] = rng.integers(60000, 70000, int(big.sum()))
    desc, total = wl.ragged_desc(rng, lens)
    desc["opcode"] = rng.choice([0x81, 0x82, 0x88, 0x89], n)
    desc["status"] = np.where(desc["opcode"] == 0x88, 1000, 0)
    return wl.random_bytes(rng, max(total, 1)), desc


def case(world, n, chunk, root=0, bad_rank=None, seed=1):
    payload, desc = ragged_job(n, seed)
    ref, ref_off = oracle.encode_batch(payload, desc)
    uid = ca.MultiGPU.unique_id()
    groups = [ca.MultiGPU.rank(0, uid, r, world) for r in range(world)]
    p = torch.from_numpy(payload).cuda()
    descs, wires, woffs = [], [], []
    for r in range(world):
        ids = shard.rank_frames(r, world, n, chunk)
        d = desc[ids]
        cap = int(ca.frame_sizes(d).sum()) if len(ids) else 0
        if r == bad_rank:
            cap //= 2
        descs.append(ca.desc_to_tensor(d, "cuda") if len(ids) else torch.empty(0, dtype=torch.uint8, device="cuda"))
        wires.append(torch.empty(max(cap, 16), dtype=torch.uint8, device="cuda"))
        woffs.append(torch.empty(len(ids) + 1, dtype=torch.int64, device="cuda"))
    out = torch.full((len(ref) + 64,), 0xA5, dtype=torch.uint8, device="cuda")
    out_off = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    result = [None] * world

    def rank_thread(r):
        try:
            torch.cuda.set_device(0)
            groups[r].encode_gather(n, chunk, [p], [descs[r]], [wires[r]], [woffs[r]], root=root,
                                    out=out if r == root else None, out_off=out_off if r == root else None)
            result[r] = 0
        except ca.WSGError as e:
            result[r] = e.code
        except Exception as e:  # noqa: BLE001 — reported, not raised, so every thread is joined
            result[r] = repr(e)

    threads = [threading.Thread(target=rank_thread, args=(r,), daemon=True) for r in range(world)]
    for t in threads:
        t.start()
    deadline = time.monotonic() + 150   # a partner that never comes fails within 60 s in the double
    for t in threads:
        t.join(timeout=max(0.0, deadline - time.monotonic()))
    hung = [r for r, t in enumerate(threads) if t.is_alive()]
    rec = dict(world=world, n=n, chunk=chunk, root=root, bad_rank=bad_rank, rc=result, hung=hung)
    if hung:   # a rank stuck in the exchange: report and leave (its handles stay open)
        print(json.dumps(dict(cases=[rec], loopback_errors=-1)), flush=True)
        os._exit(3)
    if not hung and bad_rank is None and all(x == 0 for x in result):
        got = out.cpu().numpy()
        rec["wire_ok"] = bool(np.array_equal(got[: len(ref)], ref) and (got[len(ref):] == 0xA5).all())
        rec["off_ok"] = bool(np.array_equal(out_off.cpu().numpy().view(np.uint64), ref_off))
    for g in groups:
        g.close()
    print("case %s" % json.dumps(rec), file=sys.stderr, flush=True)
    return rec


def main():
    cases = []
    if os.environ.get("WSG_RANK_JOB") == "ordering":
        # the copy-ordering check (test_mgpu_rank_form_copy_ordering, with
        # $WSG_TEST_NULL_SPIN_US set): the shape of the round-3 flake and one more
        cases.append(case(2, 9000, 1024, seed=2 * 7919 + 9000 + 1024))
        cases.append(case(3, 5000, 700, root=2, seed=3 * 7919 + 5000 + 700))
        import ctypes

        lb = ctypes.CDLL(os.environ["WSG_RCCL_LIB"])
        print(json.dumps(dict(cases=cases, loopback_errors=int(lb.loopback_rccl_errors()))), flush=True)
        return
    for world in (2, 3, 8):
        for n, chunk in ((1000, 1), (5000, 700), (9000, 1024)):
            cases.append(case(world, n, chunk, seed=world * 7919 + n + chunk))
        cases.append(case(world, 4000, 300, root=world - 1, seed=11 + world))
    cases.append(case(8, 2500, 1024, seed=5))                  # five ranks hold nothing
    for bad in (0, 1, 2):
        cases.append(case(3, 3000, 500, root=0, bad_rank=bad, seed=17))
    import ctypes

    lb = ctypes.CDLL(os.environ["WSG_RCCL_LIB"])
    print(json.dumps(dict(cases=cases, loopback_errors=int(lb.loopback_rccl_errors()))), flush=True)


if __name__ == "__main__":
    main()
