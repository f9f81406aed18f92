import sys

from .prof import main

sys.exit(main())
