import cProfile, pstats, sys, os, io
sys.argv = ["exp_h2o.py", sys.argv[1] if len(sys.argv) > 1 else "1e9", "q10"]
root = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
sys.path.insert(0, root)
src = open(os.path.join(root, "scripts/exp_h2o.py")).read()
g = {"__name__": "__main__", "__file__": os.path.join(root, "scripts/exp_h2o.py")}
# run the setup + warm queries, then profile one more q10
exec(compile(src, "exp_h2o.py", "exec"), g)
pr = cProfile.Profile()
pr.enable()
r = g["Q"]["q10"]()
g["_lib"].synchronize()
pr.disable()
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(35)
print(s.getvalue()[:9000])
