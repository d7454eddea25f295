"""debug: the round-growth self check (device best split of every leaf vs the CPU finder)"""
import json, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
import lightgbmv1_amd as lgb
from lightgbmv1_amd import _native as nat
from test_gpu_rounds import _data
os.environ["LGBM_AMD_ROUND_K"] = "8"
X, y = _data(seed=5)
p = {"objective": "binary", "verbose": -1, "device_type": "gpu", "num_leaves": 63, "max_bin": 63, "seed": 3}
for it in (1, 2, 3):
    bst = lgb.train(p, lgb.Dataset(X, y, params=p), it, keep_training_booster=True)
    res = json.loads(nat.read_string(lambda size, need, buf: nat.call(
        "LGBM_AMD_BoosterDeviceCheckSplits", bst.handle, size, need, buf), 1 << 16))
    print(it, json.dumps(res)[:1500])
