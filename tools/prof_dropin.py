import cProfile, pstats, sys, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
sys.argv = ["x", "--pods", "1000"]
import tools.bench_dropin as b
from kubernetes_amd import workload
w = workload.build("config2", n_nodes=5000, n_pods=1000)
b.run("modeler", w, 50)
pr = cProfile.Profile(); pr.enable()
rate, _ = b.run("modeler", w, 1000)
pr.disable()
print("rate", rate)
pstats.Stats(pr).sort_stats("tottime").print_stats(18)
