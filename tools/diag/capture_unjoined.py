"""Diagnostic: HIP stream-capture state after hipStreamEndCapture fails on unjoined work."""
import ctypes
import torch

hip = ctypes.CDLL("libamdhip64.so")
V = ctypes.c_void_p


def status(s):
    st = ctypes.c_int(0)
    rc = hip.hipStreamIsCapturing(V(s.cuda_stream), ctypes.byref(st))
    return rc, st.value


def end(s):
    g = V(0)
    rc = hip.hipStreamEndCapture(V(s.cuda_stream), ctypes.byref(g))
    if g.value:
        hip.hipGraphDestroy(g)
    return rc


x = torch.zeros(1024, device="cuda")
A, B = torch.cuda.Stream(), torch.cuda.Stream()
torch.cuda.synchronize()
print("begin", hip.hipStreamBeginCapture(V(A.cuda_stream), 0))
with torch.cuda.stream(A):
    x.add_(1)
B.wait_stream(A)
with torch.cuda.stream(B):
    x.add_(2)
print("status A,B", status(A), status(B))
print("end A (unjoined)", end(A))
print("status A,B after", status(A), status(B))
print("end B", end(B), "status", status(A), status(B))
# join B into A and end A again
ev = V(0)
hip.hipEventCreateWithFlags(ctypes.byref(ev), 2)
print("record B", hip.hipEventRecord(ev, V(B.cuda_stream)), "wait A", hip.hipStreamWaitEvent(V(A.cuda_stream), ev, 0))
print("end A again", end(A), "status", status(A), status(B))
print("end B again", end(B), "status", status(A), status(B))
print("last error", hip.hipGetLastError())
try:
    y = torch.empty(10, device="cuda"); y.fill_(1); torch.cuda.synchronize(); print("eager ok")
except Exception as e:
    print("eager failed:", str(e).splitlines()[0])
