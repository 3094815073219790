import cProfile, pstats, sys, time, os
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "distributed-learning-contributivity_amd"))
import numpy as np, torch
import bench
from mplc.contributivity import Contributivity
from mplc.engine import CoalitionEngine
sc = bench.build_titanic_scenario()
sc.engine = CoalitionEngine.for_scenario(sc)
def step():
    sc.coalition_values = {}
    np.random.seed(0)
    c = Contributivity(scenario=sc)
    c.compute_contributivity("Shapley values")
for _ in range(3): step()
torch.cuda.synchronize()
t=time.perf_counter()
for _ in range(10): step()
torch.cuda.synchronize()
print("ms per step", (time.perf_counter()-t)*100)
cProfile.run("for _ in range(10): step()", "/tmp/pt.out")
pstats.Stats("/tmp/pt.out").sort_stats("tottime").print_stats(25)
