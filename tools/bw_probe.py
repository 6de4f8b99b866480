import os, sys
sys.path.insert(0, "tests")
from conftest import load_cbg
cbg = load_cbg()
cbg.lib().cbg_set_device(0)
for nb in (4 << 30, 1 << 30):
    print(os.environ.get("CBG_COPY_BLOCKS_PER_CU"), nb >> 20, "MiB", round(cbg.hbm_copy_bandwidth(nb, 10), 1), flush=True)
