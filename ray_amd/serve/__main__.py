import sys

from ray_amd.serve.scripts import main

sys.exit(main())
