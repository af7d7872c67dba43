import sys

from ray_amd.scripts.scripts import main

sys.exit(main())
