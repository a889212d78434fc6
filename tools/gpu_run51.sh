cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
for v in "" "CML_FUSE_STEM_POOL=0" "CML_FUSE_DOWN_BN=0" "CML_FUSE_STEM_POOL=0 CML_FUSE_DOWN_BN=0"; do
  echo "== $v"; env $v timeout -k 10 120 python tools/diag/tiny_hist.py 2>&1 | tail -1 || exit 1
done
