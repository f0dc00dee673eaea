"""CPU restatement of the reference DSL executor -- TEST INFRASTRUCTURE ONLY.

Only tests/ (and nothing on the product path) may import this module.  It restates, independently
of the C++ executor in mscclpp_amd/csrc/host/executor.cpp:

  * plan lowering: src/core/executor/execution_plan.cc:189-231 (scratch sizes), :233-311 (load,
    message-size checks), :313-420 (channels, remote buffers), :436-605 (operations: offsets,
    sizes, tbg slicing, pipelines), :610-687 (chunk offset rules);
  * execution: src/core/include/execution_kernel.hpp handle* functions (:85-453, :509-520,
    :646-684) with the reference's sum orders -- e.g. respkt/repkt start from zero, add every
    packet source in listed order, then the local payload (:358-367); rre/rres and re/res start
    from the local source and add the other inputs in listed order (:200-214, :466-472);
  * launch state: flag = per-executor counter + 1, double scratch half chosen by flag parity
    (executor.cc:492-513).

Element arithmetic is the C oracle's oracle_reduce_words (oracle/ll_oracle.c), so fp16/bf16
clipping and NaN rules are the ones pinned by tests/golden.  All ranks run in one process: every
threadblock is a coroutine whose operations complete atomically once their inputs (packets with
the right flag, semaphore tokens, barrier arrivals) are present; a round without progress is a
deadlock and raises.
"""
import ctypes
import json
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "liboracle.so")
_L = None

OPS = {"nop", "barrier", "put", "pws", "pwsf", "get", "copy", "signal", "wait", "flush", "re", "res", "rre", "rres",
       "ppkt", "rppkt", "respkt", "cpkt", "upkt", "repkt", "recpkt", "recspkt", "rlxsignal", "rlxwait", "pipeline",
       "sem_acquire", "sem_release"}
BUF = {"i": 0, "o": 1, "s": 2}
PREDEFINED_SCRATCH = 1 << 26
DEFAULT_REUSE_SCRATCH = 1 << 27
DT_CODES = {"i32": 3, "u32": 4, "f16": 0, "f32": 2, "bf16": 1, "e4m3": 5, "e5m2": 6,  # oracle dtype codes
            "u8": 11, "b15": 12}  # e4m3b15 in the executor: T == AccumT (execution_kernel.hpp:997-1007)


def _lib():
    global _L
    if _L is None:
        _L = ctypes.CDLL(_SO)
        _L.oracle_reduce_words.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
        _L.oracle_reduce_words.restype = None
    return _L


def reduce_words(dt, op, acc, val):
    acc = np.ascontiguousarray(acc, dtype=np.uint32).copy()
    val = np.ascontiguousarray(val, dtype=np.uint32)
    if acc.size:
        _lib().oracle_reduce_words(dt, op, acc.ctypes.data, val.ctypes.data, acc.size)
    return acc


class PlanError(ValueError):
    pass


# ---------------------------------------------------------------------------------------------
# lowering
# ---------------------------------------------------------------------------------------------

class RankPlan:
    """One rank's plan at one (input_size, output_size), as execution_plan.cc builds it."""

    def __init__(self, doc, rank, input_size, output_size):
        self.doc, self.rank = doc, rank
        self.name = doc["name"]
        self.collective = doc["collective"]
        self.reuse = doc.get("reuse_resources", False)
        self.dbl = doc.get("use_double_scratch_buffer", False)
        self.align = doc.get("buffer_alignment", 16)
        self.min_msg = doc.get("min_message_size", 0)
        self.max_msg = doc.get("max_message_size", 2**64 - 1)
        self.packet = doc["protocol"] == "LL"
        self.nthreads = doc.get("num_threads_per_block", 1024)
        self.input_size, self.output_size = input_size, output_size
        gpu = doc["gpus"][rank]
        if gpu["id"] != rank:
            raise PlanError("GPU rank does not match")
        self.in_chunks, self.out_chunks, self.scr_chunks = gpu["input_chunks"], gpu["output_chunks"], gpu["scratch_chunks"]
        self._check_size()
        # channels (:313-351): a channel's tag is its ordinal among this rank's channels to that peer
        self.channels, tags = [], {}
        for ch in gpu["channels"]:
            if ch["channel_type"] != "memory":
                raise PlanError("only memory channels")
            for peer in ch["connected_to"]:
                self.channels.append((peer, tags.get(peer, 0)))
                tags[peer] = tags.get(peer, 0) + 1
        self.remote = [(rb["rank"], BUF[rb["type"]]) for rb in gpu["remote_buffers"]]
        self.sem_init = [s["init_value"] for s in gpu.get("semaphores", [])]
        self.tbs = []
        tbs = sorted(gpu["threadblocks"], key=lambda t: t["id"])
        for tb in tbs:
            chans = [c for ch in tb.get("channels", []) for c in ch["channel_ids"]]
            rem = [b for ref in tb.get("remote_buffer_refs", []) for b in ref["remote_buffer_ids"]]
            entry = {"channels": chans, "remote": rem, "ops": []}
            for o in tb["ops"]:
                entry["ops"].append(self._lower(o, rem))
                if o["name"] == "pipeline":
                    entry["ops"].extend(self._lower(i, rem) for i in o["ops"])
            self.tbs.append(entry)

    # execution_plan.cc:297-311
    def _check_size(self):
        a = self.align
        if (self.input_size % a or self.output_size % a or (self.in_chunks and (self.input_size // a) % self.in_chunks)
                or (self.out_chunks and (self.output_size // a) % self.out_chunks)):
            raise PlanError("size not aligned")
        size = self.output_size if self.collective == "allgather" else self.input_size
        if size < self.min_msg or size > self.max_msg:
            raise PlanError("size out of range")

    def calc_offset(self, size, index, slices):  # :638-644
        nel = size // self.align
        mn, rem = nel // slices, nel % slices
        return (index * mn + min(index, rem)) * self.align

    def calc_size(self, size, index, slices):  # :646-649
        return self.calc_offset(size, index + 1, slices) - self.calc_offset(size, index, slices)

    def size_and_chunks(self):  # :610-636
        if self.in_chunks and self.out_chunks:
            if self.input_size // self.in_chunks != self.output_size // self.out_chunks:
                raise PlanError("size per chunk inconsistent")
            return self.input_size, self.in_chunks
        if self.in_chunks:
            return self.input_size, self.in_chunks
        if self.out_chunks:
            return self.output_size, self.out_chunks
        raise PlanError("no chunks")

    def scratch_size(self, inp, out):  # :189-216
        if self.reuse and self.scr_chunks > 0:
            return PREDEFINED_SCRATCH
        per = (inp + self.in_chunks - 1) // self.in_chunks if self.in_chunks else (out + self.out_chunks - 1) // self.out_chunks
        size = per * self.scr_chunks * (2 if self.packet else 1)
        if self.dbl:
            size *= 2
        return (size + self.align - 1) // self.align * self.align

    def max_scratch_chunk(self, scratch):  # :218-227
        if self.scr_chunks == 0:
            return 0
        if self.dbl:
            scratch //= 2
        size = (scratch + self.scr_chunks - 1) // self.scr_chunks
        return (size + self.align - 1) // self.align * self.align

    def chunk_offset(self, chunk, btype):  # :651-663
        size, n = self.size_and_chunks()
        chunk_size = (size + n - 1) // n
        if btype == 2 and self.reuse and self.max_scratch_chunk(PREDEFINED_SCRATCH) < chunk_size:
            return chunk * self.max_scratch_chunk(PREDEFINED_SCRATCH)
        return self.calc_offset(size, chunk, n)

    def chunk_bytes(self, index, n):  # :665-669
        return self.chunk_offset(index + n, None) - self.chunk_offset(index, None)

    def upper_bound_chunk(self):  # :674-687
        if self.in_chunks:
            return (self.input_size // self.align + self.in_chunks - 1) // self.in_chunks * self.align
        return (self.output_size // self.align + self.out_chunks - 1) // self.out_chunks * self.align

    def _lower(self, o, rem):  # setupOperation :480-605
        name = o["name"]
        if name not in OPS:
            raise PlanError(f"unsupported op {name}")
        op = {"op": name, "reduce": 1 if o.get("reduce_op") == "min" else 0, "chan": list(o.get("channel_ids", [])),
              "in": [], "out": [], "barrier": [o.get("barrier_id", 0), o.get("num_threadblocks", 0)],
              "sems": list(o.get("semaphore_ids", [])), "pipeline": [0, 0, 0]}
        tb_id, tbg = 0, 1
        if "tbg_info" in o:
            tb_id, tbg = o["tbg_info"]["tb_id"], o["tbg_info"]["tbg_size"]
        for key, dst in (("src_buff", op["in"]), ("dst_buff", op["out"])):
            for b in o.get(key, []):
                if "buffer_id" in b:
                    ref = b["buffer_id"]
                    btype = self.remote[rem[ref]][1]
                else:
                    ref = BUF[b["type"]]
                    btype = ref
                off = self.chunk_offset(b["index"], btype)
                size = self.chunk_bytes(b["index"], b["size"])
                off += self.calc_offset(size, tb_id, tbg)
                size = self.calc_size(size, tb_id, tbg)
                dst.append([ref, off, size])
        if "iter_context" in o:
            unit = o["iter_context"]["unit_size"]
            n_ops = len(o["ops"])
            sizes = o["iter_context"]["num_chunks"] * self.upper_bound_chunk()
            op["pipeline"] = [(sizes + unit - 1) // unit, n_ops, unit]
        return op

    def describe(self):
        """Same shape as the C ABI's mscclppAmdExecutionPlanDescribe output."""
        return {"name": self.name, "rank": self.rank, "nthreads": self.nthreads, "packet": self.packet,
                "channels": [list(c) for c in self.channels], "remote_buffers": [list(r) for r in self.remote],
                "threadblocks": self.tbs}


# ---------------------------------------------------------------------------------------------
# execution
# ---------------------------------------------------------------------------------------------

class _Blocked(Exception):
    pass


class _Rank:
    def __init__(self, plan, inp, out, scratch_bytes):
        self.plan = plan
        self.buf = {0: inp, 1: out, 2: np.zeros(scratch_bytes, np.uint8)}


class ExecutorOracle:
    """Runs one plan on `n` simulated ranks, call after call (flags and tokens persist)."""

    def __init__(self, doc, nranks):
        self.doc, self.n = doc, nranks
        self.flag = 0
        self.tokens = {}     # (receiver, sender, tag) -> count
        self.expected = {}   # (receiver, sender, tag) -> count
        self.syncers = {}    # (rank, id) -> arrivals
        self.scratch = None  # per rank scratch arrays (allocated on first call, kept)

    def execute(self, inputs, outputs, dtype, packet="LL16", send_range=None, recv_range=None):
        """inputs/outputs: per-rank uint8 arrays (outputs may be the same objects for in-place);
        returns the per-rank (input, output, scratch) arrays after the collective."""
        dt = DT_CODES[dtype]
        plans = [RankPlan(self.doc, r, inputs[r].size, outputs[r].size) for r in range(self.n)]
        if self.scratch is None:
            self.scratch = []
            for r, p in enumerate(plans):
                sb = p.scratch_size(min(send_range or inputs[r].size, p.max_msg), min(recv_range or outputs[r].size, p.max_msg))
                self.scratch_chunk = p.max_scratch_chunk(sb)
                if p.reuse:
                    sb = DEFAULT_REUSE_SCRATCH
                self.scratch.append(np.zeros(max(sb, 256), np.uint8))
        self.flag += 1
        flag = self.flag
        ll16 = packet == "LL16"
        ranks = []
        for r in range(self.n):
            rk = _Rank(plans[r], inputs[r], outputs[r], 0)
            rk.buf[2] = self.scratch[r]
            ranks.append(rk)
        soff = (self.scratch[0].size // 2) if (plans[0].dbl and flag % 2 == 0) else 0
        sems = {r: list(plans[r].sem_init) for r in range(self.n)}
        gens = []
        for r in range(self.n):
            for t, tb in enumerate(plans[r].tbs):
                gens.append(self._run_tb(ranks, r, t, tb, dt, ll16, flag, soff, sems))
        live = list(gens)
        while live:
            progressed, nxt = False, []
            for g in live:
                try:
                    if next(g):
                        progressed = True
                    nxt.append(g)
                except StopIteration:
                    progressed = True
            live = nxt
            if live and not progressed:
                raise RuntimeError("executor oracle: deadlock (no threadblock can make progress)")
        return [(rk.buf[0], rk.buf[1], rk.buf[2]) for rk in ranks]

    # -- helpers ----------------------------------------------------------------------------
    def _run_tb(self, ranks, r, t, tb, dt, ll16, flag, soff, sems):
        ops = tb["ops"]
        i = 0
        while i < len(ops):
            op = ops[i]
            if op["op"] == "pipeline":
                n_it, n_ops, unit = op["pipeline"]
                for it in range(n_it):
                    for k in range(n_ops):
                        while not self._try(ranks, r, tb, ops[i + 1 + k], dt, ll16, flag, soff, sems, it * unit, unit):
                            yield False
                        yield True
                i += n_ops + 1
                continue
            while not self._try(ranks, r, tb, op, dt, ll16, flag, soff, sems, 0, 2**64 - 1):
                yield False
            yield True
            i += 1

    def _local(self, rk, btype, soff):
        """getBuffer (:45-56): a view starting at the buffer (scratch: at the active half)."""
        b = rk.buf[btype]
        return b[soff:] if btype == 2 else b

    def _remote(self, ranks, r, tb, ref):
        """A peer buffer from its base: non-packet operations address a peer's scratch without the
        active-half offset (memoryChannelBufferPtrs_ + offset), packet operations add it themselves."""
        peer, btype = ranks[r].plan.remote[tb["remote"][ref]]
        return ranks[peer].buf[btype]

    @staticmethod
    def _pk_ready(arr, off, n, flag, ll16):
        if n == 0:
            return True
        if ll16:
            w = arr[off:off + 16 * n].view(np.uint32).reshape(n, 4)
            return bool(np.all(w[:, 1] == flag) and np.all(w[:, 3] == flag))
        w = arr[off:off + 8 * n].view(np.uint32).reshape(n, 2)
        return bool(np.all(w[:, 1] == flag))

    @staticmethod
    def _pk_payload(arr, off, n, ll16):
        if ll16:
            return arr[off:off + 16 * n].view(np.uint32).reshape(n, 4)[:, [0, 2]].reshape(-1).copy()
        return arr[off:off + 8 * n].view(np.uint32).reshape(n, 2)[:, 0].copy()

    @staticmethod
    def _pk_write(arr, off, words, flag, ll16):
        if ll16:
            n = words.size // 2
            p = np.empty((n, 4), np.uint32)
            p[:, 0], p[:, 2] = words[0::2], words[1::2]
            p[:, 1] = p[:, 3] = flag
        else:
            n = words.size
            p = np.empty((n, 2), np.uint32)
            p[:, 0], p[:, 1] = words, flag
        arr[off:off + p.nbytes] = p.view(np.uint8).reshape(-1)

    def _try(self, ranks, r, tb, op, dt, ll16, flag, soff, sems, offset, unit):
        name = op["op"]
        rk = ranks[r]
        pay = 8 if ll16 else 4
        ins, outs = op["in"], op["out"]
        red = op["reduce"]

        def reuse_off(btype, off):  # getOffset<ReuseScratch> (:58-67)
            if rk.plan.reuse and btype == 2:
                return off % (self.scratch_chunk or 1)
            return off

        if name in ("nop", "flush"):
            return True
        if name in ("signal", "rlxsignal"):
            for c in op["chan"]:
                peer, tag = rk.plan.channels[tb["channels"][c]]
                key = (peer, r, tag)
                self.tokens[key] = self.tokens.get(key, 0) + 1
            return True
        if name in ("wait", "rlxwait"):
            keys = []
            for c in op["chan"]:
                peer, tag = rk.plan.channels[tb["channels"][c]]
                keys.append((r, peer, tag))
            if any(self.tokens.get(k, 0) < self.expected.get(k, 0) + 1 for k in keys):
                return False
            for k in keys:
                self.expected[k] = self.expected.get(k, 0) + 1
            return True
        if name == "barrier":
            sid, nblk = op["barrier"]
            key = (r, sid)
            st = self.syncers.setdefault(key, {"count": 0, "mine": {}})
            tbkey = id(tb)
            if tbkey not in st["mine"]:
                old = st["count"]
                st["count"] += 1
                st["mine"][tbkey] = (old // nblk + 1) * nblk
            if st["count"] < st["mine"][tbkey]:
                return False
            del st["mine"][tbkey]
            return True
        if name == "sem_acquire":
            if any(sems[r][s] <= 0 for s in op["sems"]):
                return False
            for s in op["sems"]:
                sems[r][s] -= 1
            return True
        if name == "sem_release":
            for s in op["sems"]:
                sems[r][s] += 1
            return True
        if name in ("put", "pws", "pwsf"):  # handlePut (:144-185)
            src = self._local(rk, ins[0][0], soff)
            for k, (ref, off, size) in enumerate(outs):
                if size <= offset:
                    continue
                n = min(size - offset, unit)
                dst = self._remote(ranks, r, tb, ref)
                peer_type = rk.plan.remote[tb["remote"][ref]][1]
                d0 = off + reuse_off(peer_type, offset)
                s0 = ins[k][1] + reuse_off(ins[k][0], offset)
                dst[d0:d0 + n] = src[s0:s0 + n]
            return True
        if name == "get":  # handleGet (:129-142), offsets exactly as the reference indexes them
            for k, (ref, off, size) in enumerate(ins):
                if size <= offset:
                    continue
                n = min(size - offset, unit)
                src = self._remote(ranks, r, tb, ref)
                peer_type = rk.plan.remote[tb["remote"][ref]][1]
                dst = self._local(rk, outs[k][0], soff)
                dst_off = outs[k][1] + reuse_off(outs[k][0], offset)
                src_off = off + reuse_off(peer_type, offset)
                dst[src_off:src_off + n] = src[dst_off:dst_off + n]
            return True
        if name == "copy":  # handleCopy (:509-520)
            if ins[0][2] <= offset:
                return True
            n = min(ins[0][2] - offset, unit)
            src = self._local(rk, ins[0][0], soff)
            dst = self._local(rk, outs[0][0], soff)
            s0 = ins[0][1] + reuse_off(ins[0][0], offset)
            d0 = outs[0][1] + reuse_off(outs[0][0], offset)
            dst[d0:d0 + n] = src[s0:s0 + n].copy()
            return True
        if name in ("rre", "rres", "re", "res"):
            if ins[0][2] <= offset:
                return True
            n = min(ins[0][2] - offset, unit) // 4 * 4
            src = self._local(rk, ins[0][0], soff)
            s0 = ins[0][1] + reuse_off(ins[0][0], offset)
            acc = src[s0:s0 + n].view(np.uint32).copy()
            for k, (ref, off, _) in enumerate(ins[1:]):
                if name in ("rre", "rres"):
                    arr = self._remote(ranks, r, tb, ref)
                    t = rk.plan.remote[tb["remote"][ref]][1]
                    o0 = off + reuse_off(t, offset)
                else:  # handleReduceSend reads local buffers (offset rule keyed on the output ref, :468)
                    arr = self._local(rk, ref, soff)
                    o0 = off + reuse_off(outs[k + 1][0] if k + 1 < len(outs) else ref, offset)
                acc = reduce_words(dt, red, acc, arr[o0:o0 + n].view(np.uint32))
            dst = self._local(rk, outs[0][0], soff)
            d0 = outs[0][1] + reuse_off(outs[0][0], offset)
            dst[d0:d0 + n] = acc.view(np.uint8)
            if name in ("rres", "res"):
                for ref, off, _ in outs[1:]:
                    arr = self._remote(ranks, r, tb, ref)
                    t = rk.plan.remote[tb["remote"][ref]][1]
                    o0 = off + reuse_off(t, offset)
                    arr[o0:o0 + n] = acc.view(np.uint8)
            return True
        if name == "ppkt":  # handlePutPackets (:262-296)
            src = self._local(rk, ins[0][0], soff)
            for k, (ref, off, _) in enumerate(outs):
                size = ins[k][2]
                npk = size // pay
                words = src[ins[k][1]:ins[k][1] + npk * pay].view(np.uint32)
                self._pk_write(self._remote(ranks, r, tb, ref), (off << 1) + soff, words, flag, ll16)
            return True
        if name == "cpkt":  # handleCopyPackets (:444-453)
            npk = ins[0][2] // pay
            src = self._local(rk, ins[0][0], soff)
            words = src[ins[0][1]:ins[0][1] + npk * pay].view(np.uint32)
            self._pk_write(self._local(rk, outs[0][0], soff), outs[0][1] << 1, words, flag, ll16)
            return True
        if name == "upkt":  # handleUnpackPackets (:428-442)
            npk = ins[0][2] // pay
            scr = rk.buf[2]
            off = soff + (ins[0][1] << 1)
            if not self._pk_ready(scr, off, npk, flag, ll16):
                return False
            words = self._pk_payload(scr, off, npk, ll16)
            dst = self._local(rk, outs[0][0], soff)
            dst[outs[0][1]:outs[0][1] + npk * pay] = words.view(np.uint8)
            return True
        if name == "rppkt":  # handleReadPutPackets (:298-337)
            npk = ins[0][2] // pay
            scr = rk.buf[2]
            off = soff + (ins[0][1] << 1)
            if not self._pk_ready(scr, off, npk, flag, ll16):
                return False
            words = self._pk_payload(scr, off, npk, ll16)
            for ref, o, _ in outs:
                self._pk_write(self._remote(ranks, r, tb, ref), soff + (o << 1), words, flag, ll16)
            return True
        if name in ("respkt", "repkt", "recspkt", "recpkt"):  # :339-426
            npk = ins[0][2] // pay
            scr = rk.buf[2]
            srcs = [soff + 2 * off for _, off, _ in ins[1:]]
            if not all(self._pk_ready(scr, o, npk, flag, ll16) for o in srcs):
                return False
            acc = np.zeros(npk * pay // 4, np.uint32)
            for o in srcs:
                acc = reduce_words(dt, red, acc, self._pk_payload(scr, o, npk, ll16))
            src = self._local(rk, ins[0][0], soff)
            s0 = ins[0][1] // pay * pay
            acc = reduce_words(dt, red, acc, src[s0:s0 + npk * pay].view(np.uint32))
            dst = self._local(rk, outs[0][0], soff)
            d0 = outs[0][1] // pay * pay
            dst[d0:d0 + npk * pay] = acc.view(np.uint8)
            first_remote = 1
            if name in ("recspkt", "recpkt"):
                self._pk_write(self._local(rk, outs[1][0], soff), 2 * outs[1][1], acc, flag, ll16)
                first_remote = 2
            if name in ("respkt", "recspkt"):
                for ref, o, _ in outs[first_remote:]:
                    self._pk_write(self._remote(ranks, r, tb, ref), soff + 2 * o, acc, flag, ll16)
            return True
        raise PlanError(f"oracle cannot run op {name}")


def load(path):
    with open(path) as f:
        return json.load(f)
