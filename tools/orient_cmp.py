import numpy as np, sys
a = np.load(sys.argv[1]); b = np.load(sys.argv[2])
print("n", len(a), len(b))
m = min(len(a), len(b))
fa = a[:m].view(np.float32); fb = b[:m].view(np.float32)
diff = np.nonzero((a[:m] != b[:m]).any(1))[0]
print("rows differing", len(diff), "first", diff[:10])
for i in diff[:8]:
    print(i, fa[i, :5], a[i, 5:], "|", fb[i, :5], b[i, 5:])
