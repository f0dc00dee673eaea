"""A buffer freed and re-allocated at the same address: does hipIpcGetMemHandle give the same handle?
(it does not, so the importers' handle-keyed cache maps the new allocation.)

    python tools/ipc_handle_probe.py
"""
import ctypes
H = ctypes.CDLL("libamdhip64.so")
vp = ctypes.c_void_p
def malloc(n):
    p = vp(); assert H.hipMalloc(ctypes.byref(p), ctypes.c_size_t(n)) == 0; return p
def handle(p):
    h = (ctypes.c_ubyte * 64)(); assert H.hipIpcGetMemHandle(h, p) == 0; return bytes(h)
H.hipSetDevice(0)
a = malloc(1 << 20); ha = handle(a); print("a", hex(a.value), ha.hex())
H.hipFree(a)
b = malloc(1 << 20); hb = handle(b); print("b", hex(b.value), hb.hex())
print("same address", a.value == b.value, "same handle", ha == hb)
