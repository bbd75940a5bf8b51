"""Same-box A/B of two builds of the package (tuning aid, GPU only): the working tree and a
second build kept under ab_old/ (a git worktree of an earlier commit, built there and copied in by
tools/make_ab_old.sh, so both libraries travel to the GPU box; delete it when done).  Each round runs every arm in its own process
(both packages are named po2_quantization_amd), alternating arms, so box drift hits both alike.

  python tools/ab_pkg.py pair      # conv_pair stage 1 (bs = 256 @224): plain chain and BasicBlock form
  python tools/ab_pkg.py bench     # bench.py's chain (no CPU baseline / extra configs)
  python tools/ab_pkg.py cifar     # bench.py's config-2 line (ResNet56 @32 chain kernels, HIP graph)
  python tools/ab_pkg.py models    # bench.py's config-3 / config-5 lines (MobileNetV2 @32, MobileViT @256)
  python tools/ab_pkg.py bench 3 PO2Q_PAIR_C32=1   # the working tree without / with an env setting
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

PAIR = r'''
import json, sys, torch
sys.path.insert(0, ".")
from po2_quantization_amd import _lib
torch.manual_seed(0)
dev = torch.device("cuda:0")
out = {}
for C, H in ((16, 224), (32, 112)):
    x = torch.relu(torch.randn(256, C, H, H, device=dev))
    w1 = torch.randn(C, C, 3, 3, device=dev) * 0.1
    w2 = torch.randn(C, C, 3, 3, device=dev) * 0.1
    ps = torch.rand(C, device=dev) + 0.5
    pb = torch.randn(C, device=dev) * 0.1
    forms = {"plain": lambda: _lib.qconv2d_pair(x, w1, w2, 4, "po2"),
             "block": lambda: _lib.qconv2d_pair(x, w1, w2, 4, "po2", post_scale1=ps, post_shift1=pb, act1="relu",
                                                post_scale2=ps, post_shift2=pb, act2="relu", residual=x)}
    for name, f in forms.items():
        for _ in range(5):
            f()
        ts = []
        for _ in range(21):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(); f(); b.record(); b.synchronize()
            ts.append(a.elapsed_time(b))
        out["C%d_%s" % (C, name)] = sorted(ts)[len(ts) // 2]
print("AB " + json.dumps(out))
'''


def run_arm(root, what, extra=None):
    env = dict(os.environ)
    env.pop("PO2Q_LIB", None)
    env.update(extra or {})
    if what == "pair":
        cmd = [sys.executable, "-c", PAIR]
    elif what == "cifar":  # the config-2 chain (ResNet56 @32, HIP graph) of bench.py's extra line
        cmd = [sys.executable, "bench.py", "--steps", "3", "--warmup", "1", "--no-cpu-baseline", "--no-models"]
    elif what == "models":  # the config-3 / config-5 lines (MobileNetV2 @32, MobileViT-XS @256, HIP graphs)
        cmd = [sys.executable, "bench.py", "--steps", "3", "--warmup", "1", "--no-cpu-baseline", "--no-cifar"]
    else:
        cmd = [sys.executable, "bench.py", "--steps", "30", "--warmup", "3", "--no-cpu-baseline", "--no-cifar",
               "--no-models"]
    p = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=600)
    if p.returncode != 0:
        raise RuntimeError("%s failed (%d): %s" % (root, p.returncode, p.stderr[-2000:]))
    for line in p.stdout.splitlines():
        if line.startswith("AB "):
            return json.loads(line[3:])
        if line.startswith("{") and '"metric"' in line:
            d = json.loads(line)
            if what == "cifar":
                c = d["config2_cifar32"]
                return {"img_s": c["value"], "ms_per_step": c["ms_per_step"],
                        "chain16_ms": c["roofline"]["avg_launch_ms"]}
            if what == "models":
                return {"c3_img_s": d["config3_mobilenet32"]["value"], "c5_img_s": d["config5_mobilevit256"]["value"]}
            return {"img_s": d["value"], "ms_per_step": d["ms_per_step"]}
    raise RuntimeError("no result from " + root)


def main():
    what = sys.argv[1] if len(sys.argv) > 1 else "pair"
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    if len(sys.argv) > 3:  # env A/B on the working tree
        k, v = sys.argv[3].split("=", 1)
        arms = {"base": (ROOT, {}), sys.argv[3]: (ROOT, {k: v})}
    else:
        arms = {"new": (ROOT, {}), "old": (os.path.join(ROOT, "ab_old"), {})}
    res = {k: [] for k in arms}
    for r in range(rounds):
        for k, (root, extra) in (arms.items() if r % 2 == 0 else reversed(list(arms.items()))):
            v = run_arm(root, what, extra)
            res[k].append(v)
            print(json.dumps({"round": r, "arm": k, **v}), flush=True)
    for k, vs in res.items():
        keys = vs[0].keys()
        med = {key: sorted(v[key] for v in vs)[len(vs) // 2] for key in keys}
        print(json.dumps({"arm": k, "median": med}), flush=True)


if __name__ == "__main__":
    main()
