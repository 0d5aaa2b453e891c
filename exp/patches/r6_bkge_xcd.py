# Candidate: r6_bk_xcd + r6_ge_xcd together.
import subprocess, sys, os
here = os.path.dirname(os.path.abspath(__file__))
for p in ("r6_bk_xcd.py", "r6_ge_xcd.py"):
    subprocess.check_call([sys.executable, os.path.join(here, p), sys.argv[1]])
