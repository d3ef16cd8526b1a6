"""Run tools/pmc_sq.sh (K_RE: kernel regex) and print tools/pmc_sq_summary.py of its output
(a python step for tools/gpu_steps.sh)."""
import os, subprocess, sys
R = os.environ.get("GRAFT_REPO_ROOT", os.getcwd())
tag = sys.argv[1] if len(sys.argv) > 1 else "sq"
rc = subprocess.call(["bash", os.path.join(R, "tools", "pmc_sq.sh"), tag])
if rc == 0:
    rc = subprocess.call([sys.executable, os.path.join(R, "tools", "pmc_sq_summary.py"), os.path.join(R, "gpurun_out", tag)])
sys.exit(rc)
