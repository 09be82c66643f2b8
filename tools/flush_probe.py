"""Where a processor flush's fixed cost goes: a C2-shaped stream pushed from host memory through a
CEP_SESSION_CARRY session in batches of `per` records, each collected (GpuCEPProcessor.flush's
cep_push_batch + cep_collect), with the host-side time of the push call and of the collect call
split, for pinned and for pageable (plain numpy) host input.

Usage: flush_probe.py [per=65536] [batches=200]
The "C loop" lines run the same loop in C (tools/flush_loop.c, built here with gcc): the C-ABI's own
cost per flush, without Python in the loop, as the JNI shim sees it.
Run under `rocprofv3 --kernel-trace --memory-copy-trace --marker-trace --stats` with KCEP_ROCTX=1
for the device-side split."""
import ctypes as C
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kafkastreams-cep_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from kcep import native as N, synth, Schema  # noqa: E402

per = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 16
nb = int(sys.argv[2]) if len(sys.argv) > 2 else 200
n = per * nb
K = max(1000, n // 100)
dev = torch.device("cuda", 0)
key, val, order = synth.c2_stream_torch(n, K, dev)
# the same records in arrival (generation) order: keys interleaved, for CEP_BATCH_ARRIVAL_ORDER
akey, aval = torch.empty_like(key), torch.empty_like(val)
akey[order] = key
aval[order] = val
ak, av = akey.cpu().pin_memory(), aval.cpu().pin_memory()
ir = synth.c2_pattern().to_ir(Schema([("value", "i32")]))
pat = N.CompiledPattern(ir)
st = torch.cuda.current_stream(dev)
pk, pv = key.cpu().pin_memory(), val.cpu().pin_memory()
hk, hv = key.cpu().numpy().copy(), val.cpu().numpy().copy()
want = None


def one_pass(sess, k_ptr, v_ptr):
    tp = tc = 0.0
    tot = 0
    for i in range(nb):
        a = i * per
        t0 = time.perf_counter()
        sess.push(per, k_ptr + 4 * a, [v_ptr + 4 * a], mem=N.MEM_HOST, stream=st.cuda_stream,
                  flags=N.BATCH_OFFSETS_MONOTONE | N.BATCH_DELIVER)
        t1 = time.perf_counter()
        out = sess.collect()
        t2 = time.perf_counter()
        tp += t1 - t0
        tc += t2 - t1
        tot += len(out["match_record"])
    return tp, tc, tot


for label, kp, vp in (("pinned", pk.data_ptr(), pv.data_ptr()), ("pageable", hk.ctypes.data, hv.ctypes.data)):
    s = N.Session(pat, per, mode=N.MODE_PROCESSOR, carry=True, max_keys=K)
    s.set_timing(False)
    one_pass(s, kp, vp)
    best = None
    for _ in range(3):
        s.state_clear()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        tp, tc, tot = one_pass(s, kp, vp)
        dt = time.perf_counter() - t0
        if best is None or dt < best[0]:
            best = (dt, tp, tc, tot)
    dt, tp, tc, tot = best
    want = tot if want is None else want
    print(f"{label:9s} per={per} batches={nb}: {dt / nb * 1e6:8.1f} us/batch  push {tp / nb * 1e6:7.1f}  "
          f"collect {tc / nb * 1e6:7.1f}  {n / dt:.3e} events/s  matches {tot} (same: {tot == want})", flush=True)
    s.close()


so = os.path.join("/tmp", "libflush_loop_%d.so" % os.getpid())
subprocess.run(["gcc", "-O2", "-shared", "-fPIC", "-o", so, os.path.join(ROOT, "tools", "flush_loop.c"),
                "-I", os.path.join(ROOT, "include"), "-L", os.path.dirname(N.LIB_PATH), "-l:libkcep.so",
                "-Wl,-rpath," + os.path.dirname(N.LIB_PATH)], check=True)
fl = C.CDLL(so)
for f in (fl.flush_loop, fl.flush_loop_pipelined):
    f.argtypes = [C.c_void_p, C.c_int64, C.c_int64, C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p,
                  C.POINTER(C.c_double)]
A = N.BATCH_ARRIVAL_ORDER
for label, kp, vp, xf, loop in (("pinned", pk.data_ptr(), pv.data_ptr(), 0, fl.flush_loop),
                                ("pageable", hk.ctypes.data, hv.ctypes.data, 0, fl.flush_loop),
                                ("pinned arrival", ak.data_ptr(), av.data_ptr(), A, fl.flush_loop),
                                ("pinned arrival pipelined", ak.data_ptr(), av.data_ptr(), A, fl.flush_loop_pipelined),
                                ("pinned grouped pipelined", pk.data_ptr(), pv.data_ptr(), 0, fl.flush_loop_pipelined)):
    s = N.Session(pat, per, mode=N.MODE_PROCESSOR, carry=True, max_keys=K)
    s.set_timing(False)
    best = None
    for _ in range(4):
        s.state_clear()
        torch.cuda.synchronize()
        o = (C.c_double * 4)()
        rc = loop(s.h, nb, per, kp, vp, N.BATCH_OFFSETS_MONOTONE | N.BATCH_DELIVER | xf, st.cuda_stream, o)
        assert rc == 0, rc
        if best is None or o[0] < best[0]:
            best = list(o)
    dt, tp, tc, tot = best
    print(f"C loop {label:25s} per={per} batches={nb}: {dt / nb:8.1f} us/batch  push {tp / nb:7.1f}  "
          f"collect {tc / nb:7.1f}  {n / (dt * 1e-6):.3e} events/s  matches {int(tot)} (same: {int(tot) == want})",
          flush=True)
    s.close()
os.unlink(so)
