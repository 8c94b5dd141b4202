"""Round-3 abort (What's weak 6): a pytest process whose FIRST HIP call came after
GPU-using child processes had exited aborted in its first runtime call.  This runs each scenario in
a fresh parent process that (optionally) imports torch without touching the GPU, runs a child to
completion, and only then makes its first HIP call (hipGetDeviceCount / hipSetDevice / hipMalloc
through libamdhip64), printing one JSON line per scenario.
Usage (GPU box): python tools/microbench/child_first_init.py"""
import json
import subprocess
import sys

CHILDREN = {
    "none": None,
    "torch_child": [sys.executable, "-c",
                    "import torch; x = torch.zeros(1, device='cuda'); torch.cuda.synchronize(); print('child ok')"],
    "hip_ctypes_child": [sys.executable, "-c",
                         "import ctypes; h = ctypes.CDLL('libamdhip64.so'); n = ctypes.c_int(0); "
                         "rc = h.hipGetDeviceCount(ctypes.byref(n)); p = ctypes.c_void_p(); "
                         "rc2 = h.hipMalloc(ctypes.byref(p), 1 << 20); h.hipFree(p); print('child ok', rc, n.value, rc2)"],
    "two_torch_children": "two",
}

PARENT = r'''
import ctypes, json, os, subprocess, sys, time
if {import_torch}:
    import torch  # no GPU call
child = {child!r}
res = {{}}
if child == "two":
    for _ in range(2):
        r = subprocess.run([sys.executable, "-c", "import torch; torch.zeros(1, device='cuda'); torch.cuda.synchronize()"],
                           capture_output=True, text=True, timeout=120)
        res.setdefault("child_rc", []).append(r.returncode)
elif child:
    r = subprocess.run(child, capture_output=True, text=True, timeout=120)
    res["child_rc"] = r.returncode
    res["child_out"] = (r.stdout + r.stderr)[-300:]
h = ctypes.CDLL("libamdhip64.so")
h.hipGetErrorString.restype = ctypes.c_char_p
n = ctypes.c_int(-1)
rc = h.hipGetDeviceCount(ctypes.byref(n))
res["count_rc"] = rc
res["count_err"] = h.hipGetErrorString(rc).decode()
res["count"] = n.value
rc = h.hipSetDevice(0)
res["set_rc"] = h.hipGetErrorString(rc).decode()
p = ctypes.c_void_p()
rc = h.hipMalloc(ctypes.byref(p), 1 << 20)
res["malloc"] = h.hipGetErrorString(rc).decode()
res["env"] = {{k: os.environ.get(k) for k in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES",
                                            "GPU_DEVICE_ORDINAL", "HSA_ENABLE_IPC_MODE_LEGACY")}}
print(json.dumps(res))
'''


def main():
    for import_torch in (False, True):
        for name, child in CHILDREN.items():
            code = PARENT.format(import_torch=import_torch, child=child)
            r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
            line = r.stdout.strip().splitlines()[-1] if r.stdout.strip() else r.stderr[-500:]
            print(json.dumps({"scenario": name, "parent_imports_torch": import_torch, "rc": r.returncode,
                              "result": line}), flush=True)


if __name__ == "__main__":
    main()
