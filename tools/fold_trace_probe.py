import sys; sys.path.insert(0,'/root/repo')
import numpy as np, implisolid_amd as I
rng = np.random.default_rng(1)
e = (0.0144 * (0.5 + rng.uniform(size=30000))).astype(np.float32)
print(I.debug_fold(e))
