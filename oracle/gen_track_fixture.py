"""TEST INFRASTRUCTURE: the Highway map table (PointAndTangent, halfWidth, lane) as a data fixture,
so runs that may not import oracle/ (bench.py's GPU leg) can build the reference's N = 125 case.
Made from oracle/lpv_ref.Track.build("Highway"), the restatement of Map
(planner/lib/plan_lib/mapManager/track_initialization.py) pinned against the reference's own
map goldens in tests/test_oracle_lpv.py.  Writes tests/golden/track_highway.npz."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import lpv_ref as L  # noqa: E402

if __name__ == "__main__":
    tr = L.Track.build("Highway")
    path = os.path.join(ROOT, "tests", "golden", "track_highway.npz")
    np.savez_compressed(path, PointAndTangent=tr.PointAndTangent, halfWidth=np.asarray(tr.halfWidth, float),
                        lane=np.array(tr.lane), TrackLength=np.asarray(tr.TrackLength, float))
    print("wrote", path)
