import sys

from ray_amd.rllib.scripts import main

sys.exit(main())
