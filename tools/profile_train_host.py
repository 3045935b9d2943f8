import cProfile, pstats, sys, io, os
sys.argv = ["bench_train.py", "--n", "100000", "--ids", "10000", "--n-cpu", "50", "--predict", "256"]
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo") + "/tools")
import bench_train
pr = cProfile.Profile()
pr.enable()
bench_train.main()
pr.disable()
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(45)
print(s.getvalue()[:12000])
