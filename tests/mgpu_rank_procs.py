"""The RCCL rank-per-process form of wsg_mgpu_encode_gather at world > 1 over
the REAL RCCL, one process per rank, every rank on the one GPU of the box.

RCCL refuses two ranks of one host on one device ("Duplicate GPU detected":
it compares host hash and PCI bus id).  Each rank here gets its own
$NCCL_HOSTID, so RCCL sees `world` single-GPU hosts and connects them with
its network transport (sockets over the loopback interface) instead of xGMI
P2P: the bytes take another road, but every call the product makes —
ncclCommInitRank from wsg_mgpu_unique_id's id, the status and chunk-size
ncclAllGather rounds, the grouped per-chunk ncclSend/ncclRecv into the root —
runs in RCCL itself, process against process (the loopback test double of
tests/mgpu_rank_job.py stands in for RCCL; this does not).

Parent: `python tests/mgpu_rank_procs.py [--big]` (touches no GPU) runs every
case as `world` child processes of this script and prints one JSON line
{"cases": [...]}; a child: `--child RANK WORLD N CHUNK ROOT BAD SEED DIR`.
Rank 0 makes the id (its process hosts RCCL's bootstrap root) and hands it
to the others through DIR.  The root checks its wire and offsets against the
oracle's encode of the whole job; every rank reports its return code.
"""
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def child(rank, world, n, chunk, root, bad, seed, d):
    import numpy as np
    import torch

    import oracle
    import cppserver_amd as ca
    from cppserver_amd import shard
    from cppserver_amd import workloads as wl
    from tests.mgpu_rank_job import ragged_job

    if seed < 0:   # C5-shape frames: 16 KiB payloads, a random key each
        ids = np.arange(n)
        payload, desc = wl.c5_payload_np(ids, 16384), wl.c5_desc(ids, 16384)
    else:
        payload, desc = ragged_job(n, seed)
    uid_path = os.path.join(d, "uid")
    if rank == 0:
        uid = ca.MultiGPU.unique_id()
        with open(uid_path + ".tmp", "wb") as f:
            f.write(uid)
        os.rename(uid_path + ".tmp", uid_path)
    else:
        deadline = time.monotonic() + 60
        while not os.path.exists(uid_path):
            if time.monotonic() > deadline:
                raise SystemExit("no id from rank 0")
            time.sleep(0.01)
        with open(uid_path, "rb") as f:
            uid = f.read()
    torch.cuda.set_device(0)
    g = ca.MultiGPU.rank(0, uid, rank, world)
    ids = shard.rank_frames(rank, world, n, chunk)
    dsc = desc[ids]
    cap = int(ca.frame_sizes(dsc).sum()) if len(ids) else 0
    if rank == bad:
        cap //= 2
    p = torch.from_numpy(payload).cuda()
    dt = ca.desc_to_tensor(dsc, "cuda") if len(ids) else torch.empty(0, dtype=torch.uint8, device="cuda")
    w = torch.empty(max(cap, 16), dtype=torch.uint8, device="cuda")
    wo = torch.empty(len(ids) + 1, dtype=torch.int64, device="cuda")
    out = out_off = ref = None
    if rank == root:
        total = int(ca.frame_sizes(desc).sum())
        out = torch.full((total + 64,), 0xA5, dtype=torch.uint8, device="cuda")
        out_off = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    rec = dict(rank=rank)
    try:
        enc_ms, gat_ms = g.encode_gather(n, chunk, [p], [dt], [w], [wo], root=root, out=out, out_off=out_off)
        rec.update(rc=0, encode_ms=round(enc_ms, 3), gather_ms=round(gat_ms, 3))
    except ca.WSGError as e:
        rec["rc"] = e.code
    if rank == root and rec["rc"] == 0:
        if seed < 0:   # the whole job is too big for the oracle here: every frame's header/key, sampled frames
            ref, ref_off = oracle.encode_batch(payload[: 4096 * 16384], desc[:4096])
            got = out[: len(ref)].cpu().numpy()
            offs = out_off.cpu().numpy().view(np.uint64)
            rec["wire_ok"] = bool(np.array_equal(got, ref))
            rec["off_ok"] = bool(np.array_equal(offs, np.arange(n + 1, dtype=np.uint64) * (16384 + 8)))
            rec["bytes"] = int(out.numel() - 64)
        else:
            ref, ref_off = oracle.encode_batch(payload, desc)
            got = out.cpu().numpy()
            rec["wire_ok"] = bool(np.array_equal(got[: len(ref)], ref) and (got[len(ref):] == 0xA5).all())
            rec["off_ok"] = bool(np.array_equal(out_off.cpu().numpy().view(np.uint64), ref_off))
    g.close()
    print("RESULT " + json.dumps(rec), flush=True)


def run_case(world, n, chunk, root=0, bad=None, seed=1, timeout=150):
    d = tempfile.mkdtemp(prefix="wsg_rank_")
    procs = []
    log_dir = os.path.join(ROOT, "gpurun_out", "rank_procs")
    os.makedirs(log_dir, exist_ok=True)
    for r in range(world):
        env = dict(os.environ, NCCL_HOSTID="wsg-rank-%d" % r, NCCL_SOCKET_IFNAME="lo", NCCL_IB_DISABLE="1",
                   NCCL_DEBUG=os.environ.get("NCCL_DEBUG", "WARN"))
        log = open(os.path.join(log_dir, "w%d_n%d_c%d_r%d_b%s_rank%d.log" % (world, n, chunk, root, bad, r)), "w")
        procs.append((subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__), "--child", str(r), str(world),
                                        str(n), str(chunk), str(root), str(-1 if bad is None else bad), str(seed), d],
                                       stdout=subprocess.PIPE, stderr=log, text=True, env=env, start_new_session=True),
                      log))
    deadline = time.monotonic() + timeout
    ranks, hung = [None] * world, []
    for r, (pr, log) in enumerate(procs):
        try:
            out, _ = pr.communicate(timeout=max(1.0, deadline - time.monotonic()))
            for line in out.splitlines():
                if line.startswith("RESULT "):
                    ranks[r] = json.loads(line[7:])
            if ranks[r] is None:
                ranks[r] = dict(rank=r, exit=pr.returncode)
        except subprocess.TimeoutExpired:
            hung.append(r)
        log.close()
    for r in hung:   # the whole group of a stuck rank, by its own process group id
        pr = procs[r][0]
        try:
            os.killpg(pr.pid, 9)
        except ProcessLookupError:
            pass
        pr.wait()
    rec = dict(world=world, n=n, chunk=chunk, root=root, bad_rank=bad, seed=seed, hung=hung, ranks=ranks)
    print("case " + json.dumps(rec), file=sys.stderr, flush=True)
    return rec


def main():
    big = "--big" in sys.argv
    cases = []
    if "--ordering" in sys.argv:   # test_mgpu_rank_form_copy_ordering ($WSG_TEST_NULL_SPIN_US set)
        cases.append(run_case(2, 9000, 1024, seed=2 * 7919 + 9000 + 1024))
        print(json.dumps(dict(cases=cases)), flush=True)
        return
    for world in (2, 3):
        for n, chunk in ((1000, 1), (5000, 700), (9000, 1024)):
            cases.append(run_case(world, n, chunk, seed=world * 7919 + n + chunk))
            if cases[-1]["hung"]:
                break
        cases.append(run_case(world, 4000, 300, root=world - 1, seed=11 + world))
    cases.append(run_case(3, 3000, 500, root=0, bad=1, seed=17))
    if big:   # C5-shape frames at world 2: 64 Ki frames x 16 KiB (1 GiB of payload); world 4
        cases.append(run_case(2, 65536, 1024, seed=-1, timeout=240))
        cases.append(run_case(4, 9000, 1024, root=3, seed=4 * 7919 + 10024))
        cases.append(run_case(4, 5000, 700, root=0, bad=2, seed=23))
    print(json.dumps(dict(cases=cases)), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        a = sys.argv[2:]
        child(int(a[0]), int(a[1]), int(a[2]), int(a[3]), int(a[4]), int(a[5]), int(a[6]), a[7])
    else:
        main()
