"""Why the device decoder declines a file (experiments): gbam.decode in both modes, last_error."""
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import torch  # noqa: E402

from sctools_amd import gbam  # noqa: E402

for path in sys.argv[1:]:
    for mode in ("cell", "gene"):
        got = gbam.decode(path, mode, torch.device("cuda", 0))
        print(path, mode, "ok" if got is not None else "declined: " + gbam.last_error())
