from .gpu_exporter import main

main()
