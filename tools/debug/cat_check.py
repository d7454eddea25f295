"""debug: one-split-per-step with a categorical feature -- device best split of every leaf vs
the CPU finder on the device histograms (LGBM_AMD_BoosterDeviceCheckSplits)"""
import json, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
import lightgbmv1_amd as lgb
from lightgbmv1_amd import _native as nat
from test_gpu_rounds import _data
os.environ["LGBM_AMD_ROUND_K"] = sys.argv[1] if len(sys.argv) > 1 else "1"
X, y = _data()
for leaves in (3, 4, 5, 31):
    p = {"objective": "binary", "verbose": -1, "device_type": "gpu", "num_leaves": leaves, "max_bin": 63, "seed": 11}
    bst = lgb.train(p, lgb.Dataset(X, y, params=p, categorical_feature=[9]), 1, keep_training_booster=True)
    res = json.loads(nat.read_string(lambda size, need, buf: nat.call(
        "LGBM_AMD_BoosterDeviceCheckSplits", bst.handle, size, need, buf), 1 << 18))
    t = bst.dump_model()["tree_info"][0]
    print("leaves", leaves, "->", t["num_leaves"], json.dumps(res)[:3000], flush=True)
