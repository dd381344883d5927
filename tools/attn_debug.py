import os, sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "light-whisper_amd"))
import torch
from qasr import _lib
L = _lib.load()
dev = torch.device("cuda:0")

def run(hd, nh, nkv, starts, lens, dense, seed=1, vmode="rand", qmode="rand"):
    rng = np.random.default_rng(seed)
    slots = int(max(s + n for s, n in zip(starts, lens))) + 5
    k = rng.standard_normal((slots, nkv * hd)).astype(np.float16)
    v = rng.standard_normal((slots, nkv * hd)).astype(np.float16)
    if vmode == "keyid":
        v[:] = (np.arange(slots)[:, None] * 0.01).astype(np.float16)
    elif vmode == "ones":
        v[:] = 1
    elif vmode == "onehot":
        v[:] = 0
        v[int(os.environ.get("HOT", "0")), :] = 1
    q = rng.standard_normal((len(starts), nh * hd)).astype(np.float16)
    if qmode == "zero":
        q[:] = 0
    st, ln = np.asarray(starts, np.int32), np.asarray(lens, np.int32)
    rows = len(starts)
    t = [torch.from_numpy(a).to(dev) for a in (q, k, v, st, ln)]
    o = torch.zeros(rows, nh * hd, device=dev)
    oq = torch.zeros(rows, nh * hd, dtype=torch.int8, device=dev)
    od = torch.zeros(rows, nh * hd // 32, device=dev)
    _lib.check(L.qasr_op_attention_dense(t[0].data_ptr(), nh * hd, t[1].data_ptr(), t[2].data_ptr(), nkv * hd,
                                         t[3].data_ptr(), t[4].data_ptr(), rows, nh, nkv, hd, 1 / np.sqrt(hd),
                                         o.data_ptr(), oq.data_ptr(), od.data_ptr(), int(dense), None))
    torch.cuda.synchronize()
    oh = o.cpu().numpy()
    ref = np.zeros_like(oh, dtype=np.float64)
    for r in range(rows):
        for h in range(nh):
            g = h // (nh // nkv)
            kk = k[st[r]:st[r] + ln[r], g * hd:(g + 1) * hd].astype(np.float64)
            vv = v[st[r]:st[r] + ln[r], g * hd:(g + 1) * hd].astype(np.float64)
            s = kk @ q[r, h * hd:(h + 1) * hd].astype(np.float64) / np.sqrt(hd)
            p = np.exp(s - s.max())
            ref[r, h * hd:(h + 1) * hd] = p @ vv / p.sum()
    err = np.abs(oh - ref)
    return err.max(), oh, ref

for vm in ["ones"] + [f"onehot{j}" for j in range(6)]:
    if vm.startswith("onehot"):
        os.environ["HOT"] = vm[6:]
        vm2 = "onehot"
    else:
        vm2 = vm
    e, oh, ref = run(128, 1, 1, [0], [5], True, vmode=vm2, qmode="zero")
    print(vm, "got", oh[0, :3], oh[0, 16:18], "want", ref[0, :3])
