import cProfile, pstats, sys, io
sys.argv = ["host_prep_profile.py", "--cells", "10000"]
sys.path.insert(0, "tools")
import host_prep_profile
pr = cProfile.Profile(); pr.enable()
host_prep_profile.main()
pr.disable()
s = io.StringIO(); pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(25); print(s.getvalue()[:6000])
