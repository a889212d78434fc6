#!/usr/bin/env python3
"""MIOpen tuning of every ResNet-50 convolution that MIOpen runs in the benchmark step (bf16 NHWC):
forward, data gradient and weight gradient of each unique shape, biggest first. --mode search is
exhaustive (MIOPEN_FIND_ENFORCE=SEARCH_DB_UPDATE); --mode find records MIOpen's normal find (what
`torch.backends.cudnn.benchmark` does on first use) for a new batch size. The user db is copied
to --out after every shape, so a run cut short keeps what it tuned; --db seeds the run with an
earlier (partial) db.

  python tools/miopen_tune.py --out gpurun_out/miopen_search [--db tuning/miopen_search] \\
      [--budget 1000]
"""
import argparse
import os
import shutil
import sys
import tempfile
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def conv_shapes(batch):
    """(cin, h, w, cout, k, stride, pad) of every nn.Conv2d of resnet50 except the stem."""
    import torch
    from consensusml_amd.models.resnet import resnet50
    m = resnet50()
    seen, shapes = set(), []

    def pre(mod, inp):
        x = inp[0]
        key = (mod.in_channels, x.shape[2], x.shape[3], mod.out_channels, mod.kernel_size[0],
               mod.stride[0], mod.padding[0])
        if mod.kernel_size[0] != 7 and key not in seen:
            seen.add(key)
            shapes.append(key)
    for mod in m.modules():
        if isinstance(mod, torch.nn.Conv2d):
            mod.register_forward_pre_hook(pre)
    with torch.no_grad():
        m(torch.randn(1, 3, 224, 224))
    return shapes


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--db", default=None, help="seed user-db directory")
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--only", nargs="*", default=None,
                    help="shape keys cin x h x w x cout x k x stride x pad to tune (default: all)")
    ap.add_argument("--budget", type=float, default=1000.0, help="seconds; stop starting shapes after")
    ap.add_argument("--mode", choices=["search", "find"], default="search",
                    help="search: exhaustive (SEARCH_DB_UPDATE); find: MIOpen's normal find only")
    a = ap.parse_args()
    work = tempfile.mkdtemp(prefix="cml_miopen_search_")
    if a.db and os.path.isdir(a.db):
        for f in os.listdir(a.db):
            shutil.copy(os.path.join(a.db, f), work)
    os.environ["MIOPEN_USER_DB_PATH"] = work
    if a.mode == "search":
        os.environ["MIOPEN_FIND_ENFORCE"] = "SEARCH_DB_UPDATE"
        os.environ["MIOPEN_FIND_MODE"] = "NORMAL"
    for v in ("FWD", "BWD", "WRW"):
        os.environ[f"MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_{v}"] = "0"
    import torch
    import torch.nn.functional as F
    torch.backends.cudnn.benchmark = True
    dev = torch.device("cuda")
    shapes = conv_shapes(a.batch)
    shapes.sort(key=lambda s: -(s[0] * s[3] * s[4] * s[4] * s[1] * s[2] / s[5] ** 2))
    done = set(open(os.path.join(a.db, "done.txt")).read().split()) if a.db and os.path.exists(
        os.path.join(a.db, "done.txt")) else set()
    done = {d for d in done if d.startswith(f"b{a.batch}:")}
    t0 = time.time()
    alive = [True]

    def beat():
        while alive[0]:
            time.sleep(30)
            print(f"  ... {time.time() - t0:.0f} s", flush=True)
    threading.Thread(target=beat, daemon=True).start()
    os.makedirs(a.out, exist_ok=True)
    for s in shapes:
        key = f"b{a.batch}:" + "x".join(map(str, s))
        if a.only and "x".join(map(str, s)) not in a.only:
            continue
        if key in done:
            continue
        if time.time() - t0 > a.budget:
            print("budget reached", flush=True)
            break
        cin, h, w, cout, k, st, p = s
        ts = time.time()
        x = torch.randn(a.batch, cin, h, w, device=dev, dtype=torch.bfloat16).contiguous(
            memory_format=torch.channels_last).requires_grad_(True)
        wt = (torch.randn(cout, cin, k, k, device=dev) * 0.05).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last).requires_grad_(True)
        y = F.conv2d(x, wt, None, st, p)
        y.backward(torch.randn_like(y))
        torch.cuda.synchronize()
        done.add(key)
        for f in os.listdir(work):
            shutil.copy(os.path.join(work, f), a.out)
        with open(os.path.join(a.out, "done.txt"), "w") as fh:
            fh.write("\n".join(sorted(done)) + "\n")
        print(f"{key}: {time.time() - ts:.1f} s", flush=True)
        del x, wt, y
    alive[0] = False
    print(f"tuned {len(done)} / {len(shapes)} shapes in {time.time() - t0:.0f} s", flush=True)


if __name__ == "__main__":
    main()
