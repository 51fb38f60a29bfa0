"""Launch scripts (reference spark-submit-with-bigdl.sh & co): syntax and the command they build."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCRIPTS = ["run-with-bigdl.sh", "python-with-bigdl.sh", "jupyter-with-bigdl.sh", "run-example.sh", "make-dist.sh"]


def test_scripts_parse():
    for s in SCRIPTS:
        subprocess.run(["bash", "-n", os.path.join(ROOT, "scripts", s)], check=True)


def test_run_with_bigdl_dry_run():
    out = subprocess.run([os.path.join(ROOT, "scripts", "run-with-bigdl.sh"), "-n", "8", "--dry-run", "bench.py",
                          "--gpus", "8"], check=True, capture_output=True, text=True).stdout.strip()
    assert out == ("python3 -m torch.distributed.run --nnodes 1 --node-rank 0 --nproc-per-node 8 "
                   "--master-addr 127.0.0.1 --master-port 29500 bench.py --gpus 8")


def test_python_with_bigdl_imports_package():
    out = subprocess.run([os.path.join(ROOT, "scripts", "python-with-bigdl.sh"), "-c",
                          "import bigdl_amd, os; print(os.environ['HSA_ENABLE_IPC_MODE_LEGACY'])"],
                         check=True, capture_output=True, text=True, cwd="/tmp").stdout.strip()
    assert out.endswith("0")
