"""Phase-stamp report of the LDS-DMA conv kernel (diagnostic build: `make -C
po2_quantization_amd/csrc stamps`).  Prints, per layer config, the mean cycles
per work item per wave spent in each phase.  GPU only; timings of this build
are not representative -- read the shares."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CONFIGS = [  # (shape, PO2Q_X3P_WAVES, PO2Q_X3P_TILE)
    ("16,224,16,3,1,1", None, None),
    ("16,224,16,3,1,1", "8", "2,8,32,2"),
    ("16,224,16,3,1,1", "4", "2,4,32,2"),
    ("32,112,32,3,1,1", "8", "2,16,16,0"),
    ("64,56,64,3,1,1", "4", "4,8,32,0"),
]


def main():
    env0 = dict(os.environ, PO2Q_LIB=os.path.join(ROOT, "po2_quantization_amd", "lib_stamps", "libpo2q.so"),
                PO2Q_STAMPS="1")
    for shape, waves, tile in CONFIGS:
        env = dict(env0)
        if waves:
            env["PO2Q_X3P_WAVES"] = waves
        if tile:
            env["PO2Q_X3P_TILE"] = tile
        print("== shape %s waves %s tile %s" % (shape, waves, tile), flush=True)
        r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "prof_layer.py"), "--shape", shape,
                            "--iters", "2"], env=env, capture_output=True, text=True, timeout=300)
        print(r.stdout.strip())
        print("\n".join(l for l in r.stderr.splitlines() if "po2q stamps" in l or l.startswith("  ")), flush=True)
        if r.returncode:
            print("rc", r.returncode, r.stderr[-2000:])
            return r.returncode
    return 0


if __name__ == "__main__":
    sys.exit(main())
