import os, sys
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "tests"))
from test_mf_tiled_gpu import _train
for lv in ("3", "4"):
    os.environ["FPS_TILE_PARTITION_LEVELS"] = lv
    for rep in range(2):
        b0, a0, _ = _train(False)
        b1, a1, _ = _train(True)
        print(f"levels={lv} rep={rep} sync={a0:.5f} prefetch={a1:.5f}", flush=True)
