"""Generate the execution-plan fixtures used by the executor tests.

The plans use the reference's JSON plan format (the one its DSL emits and
src/core/executor/execution_plan.cc parses); this script is this repo's own generator of three
AllReduce algorithms over memory channels:

  allreduce_pkt_n{N}.json    LL protocol, all-pairs: ppkt every peer's chunk into its scratch,
                             respkt my chunk (sum of the peers' packets + mine, sent back as
                             packets), upkt the other chunks; T threadblocks split every chunk
                             with tbg_info.  Same operation mix as the reference's 2-rank
                             allreduce_packet plan.
  allreduce_rres_n{N}.json   Simple protocol: relaxed handshake, rres (read the peers' chunk,
                             reduce, write the result into every rank's input), then a
                             signal/wait so no rank leaves early.  Same operation mix as the
                             reference's allreduce plan.
  allreduce_put_n{N}.json    Simple protocol through scratch: put my copy of chunk q into rank q's
                             scratch, signal/wait, re (my chunk + the scratch copies), put the
                             result into every peer's output, then a workgroup barrier and a
                             semaphore hand-off between the threadblocks; exercises put, re, copy,
                             barrier, sem_acquire/sem_release and pipeline.

Run:  python tests/golden/plans/make_plans.py   (rewrites the .json files next to it)
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))


def _common(name, protocol, gpus, nthreads=1024, double=False, inplace=True):
    return {"name": name, "collective": "allreduce", "protocol": protocol, "inplace": inplace,
            "reuse_resources": False, "gpus": gpus, "num_threads_per_block": nthreads,
            "use_double_scratch_buffer": double, "buffer_alignment": 16, "min_message_size": 0,
            "max_message_size": 2**64 - 1}


def _tbg(op, t, T):
    if T > 1:
        op["tbg_info"] = {"tb_id": t, "tbg_size": T}
    return op


def allreduce_pkt(n, T=2, nthreads=512):
    gpus = []
    for r in range(n):
        peers = [q for q in range(n) if q != r]
        # remote buffer k = peer peers[k]'s scratch; channel k = peer peers[k]
        tbs = []
        for t in range(T):
            ops = []
            ops.append(_tbg({"name": "ppkt", "src_buff": [{"type": "i", "index": q, "size": 1} for q in peers],
                             "dst_buff": [{"buffer_id": k, "index": r, "size": 1} for k, _ in enumerate(peers)],
                             "channel_type": "memory"}, t, T))
            ops.append(_tbg({"name": "respkt",
                             "src_buff": [{"type": "i", "index": r, "size": 1}] +
                                         [{"type": "s", "index": q, "size": 1} for q in peers],
                             "dst_buff": [{"type": "i", "index": r, "size": 1}] +
                                         [{"buffer_id": k, "index": n + r, "size": 1} for k, _ in enumerate(peers)],
                             "channel_type": "memory", "reduce_op": "sum"}, t, T))
            for q in peers:
                ops.append(_tbg({"name": "upkt", "src_buff": [{"type": "s", "index": n + q, "size": 1}],
                                 "dst_buff": [{"type": "i", "index": q, "size": 1}]}, t, T))
            tbs.append({"id": t, "ops": ops,
                        "channels": [{"channel_type": "memory", "channel_ids": list(range(len(peers)))}],
                        "remote_buffer_refs": [{"access_channel_type": "memory",
                                                "remote_buffer_ids": list(range(len(peers)))}]})
        gpus.append({"id": r, "input_chunks": n, "output_chunks": n, "scratch_chunks": 2 * n, "threadblocks": tbs,
                     "channels": [{"channel_type": "memory", "connected_to": peers}],
                     "remote_buffers": [{"rank": q, "type": "s", "access_channel_types": ["memory"]} for q in peers],
                     "semaphores": []})
    return _common(f"allreduce_pkt_n{n}", "LL", gpus, nthreads=nthreads, double=True)


def allreduce_rres(n, per_rank_tbs=2, nthreads=512):
    """Chunks: n * per_rank_tbs; rank r owns chunks [r*P, (r+1)*P), one threadblock per chunk."""
    P = per_rank_tbs
    gpus = []
    for r in range(n):
        peers = [q for q in range(n) if q != r]
        # channels: for every threadblock one channel to every peer (channel id = t*(n-1)+k)
        conn = []
        for _t in range(P):
            conn.extend(peers)
        tbs = []
        for t in range(P):
            chunk = r * P + t
            chans = [t * (n - 1) + k for k in range(n - 1)]
            local_ids = list(range(n - 1))
            ops = [
                {"name": "rlxsignal", "channel_ids": local_ids, "channel_type": "memory"},
                {"name": "rlxwait", "channel_ids": local_ids, "channel_type": "memory"},
                {"name": "nop"},
                {"name": "rres",
                 "src_buff": [{"type": "i", "index": chunk, "size": 1}] +
                             [{"buffer_id": k, "index": chunk, "size": 1} for k in range(n - 1)],
                 "dst_buff": [{"type": "i", "index": chunk, "size": 1}] +
                             [{"buffer_id": k, "index": chunk, "size": 1} for k in range(n - 1)],
                 "channel_type": "memory", "reduce_op": "sum"},
                {"name": "nop"},
                {"name": "signal", "channel_ids": local_ids, "channel_type": "memory"},
                {"name": "wait", "channel_ids": local_ids, "channel_type": "memory"},
            ]
            tbs.append({"id": t, "ops": ops, "channels": [{"channel_type": "memory", "channel_ids": chans}],
                        "remote_buffer_refs": [{"access_channel_type": "memory", "remote_buffer_ids": list(range(n - 1))}]})
        gpus.append({"id": r, "input_chunks": n * P, "output_chunks": n * P, "scratch_chunks": 0, "threadblocks": tbs,
                     "channels": [{"channel_type": "memory", "connected_to": conn}],
                     "remote_buffers": [{"rank": q, "type": "i", "access_channel_types": ["memory"]} for q in peers],
                     "semaphores": []})
    return _common(f"allreduce_rres_n{n}", "Simple", gpus, nthreads=nthreads)


def allreduce_put(n, nthreads=256, unit=4096):
    """Out-of-place.  tb0: puts + reduction; tb1: waits on tb0 through a semaphore, then copies the
    reduced own chunk into the output in a pipeline of `unit`-byte steps.  Remote buffers: peers'
    scratch (put targets) and peers' outputs (result targets)."""
    gpus = []
    for r in range(n):
        peers = [q for q in range(n) if q != r]
        scr = list(range(n - 1))              # remote buffer ids: scratch of peers[k]
        outs = list(range(n - 1, 2 * (n - 1)))  # remote buffer ids: output of peers[k]
        tb0 = [
            {"name": "put", "src_buff": [{"type": "i", "index": q, "size": 1} for q in peers],
             "dst_buff": [{"buffer_id": k, "index": r, "size": 1} for k in range(n - 1)], "channel_type": "memory"},
            {"name": "nop"},
            {"name": "signal", "channel_ids": list(range(n - 1)), "channel_type": "memory"},
            {"name": "wait", "channel_ids": list(range(n - 1)), "channel_type": "memory"},
            {"name": "nop"},
            {"name": "re", "src_buff": [{"type": "i", "index": r, "size": 1}] +
                                       [{"type": "s", "index": q, "size": 1} for q in peers],
             "dst_buff": [{"type": "s", "index": r, "size": 1}], "reduce_op": "sum"},
            {"name": "put", "src_buff": [{"type": "s", "index": r, "size": 1} for _ in peers],
             "dst_buff": [{"buffer_id": n - 1 + k, "index": r, "size": 1} for k in range(n - 1)],
             "channel_type": "memory"},
            {"name": "sem_release", "semaphore_ids": [0]},
            {"name": "barrier", "barrier_id": 0, "num_threadblocks": 2},
            {"name": "signal", "channel_ids": list(range(n - 1)), "channel_type": "memory"},
            {"name": "wait", "channel_ids": list(range(n - 1)), "channel_type": "memory"},
        ]
        tb1 = [
            {"name": "sem_acquire", "semaphore_ids": [0]},
            {"name": "pipeline", "iter_context": {"unit_size": unit, "num_chunks": 1},
             "ops": [{"name": "copy", "src_buff": [{"type": "s", "index": r, "size": 1}],
                      "dst_buff": [{"type": "o", "index": r, "size": 1}]}]},
            {"name": "barrier", "barrier_id": 0, "num_threadblocks": 2},
        ]
        gpus.append({"id": r, "input_chunks": n, "output_chunks": n, "scratch_chunks": n,
                     "threadblocks": [
                         {"id": 0, "ops": tb0, "channels": [{"channel_type": "memory", "channel_ids": list(range(n - 1))}],
                          "remote_buffer_refs": [{"access_channel_type": "memory", "remote_buffer_ids": scr + outs}]},
                         {"id": 1, "ops": tb1}],
                     "channels": [{"channel_type": "memory", "connected_to": peers}],
                     "remote_buffers": [{"rank": q, "type": "s", "access_channel_types": ["memory"]} for q in peers] +
                                       [{"rank": q, "type": "o", "access_channel_types": ["memory"]} for q in peers],
                     "semaphores": [{"init_value": 0}]})
    return _common(f"allreduce_put_n{n}", "Simple", gpus, nthreads=nthreads, inplace=False)


PLANS = {
    "allreduce_pkt_n2.json": lambda: allreduce_pkt(2, T=2),
    "allreduce_pkt_n4.json": lambda: allreduce_pkt(4, T=2),
    "allreduce_pkt_n8.json": lambda: allreduce_pkt(8, T=4),
    "allreduce_rres_n2.json": lambda: allreduce_rres(2, per_rank_tbs=4),
    "allreduce_rres_n4.json": lambda: allreduce_rres(4, per_rank_tbs=2),
    "allreduce_put_n2.json": lambda: allreduce_put(2),
    "allreduce_put_n4.json": lambda: allreduce_put(4),
}


def main():
    for fname, fn in PLANS.items():
        with open(os.path.join(HERE, fname), "w") as f:
            json.dump(fn(), f, indent=1)
            f.write("\n")


if __name__ == "__main__":
    main()
