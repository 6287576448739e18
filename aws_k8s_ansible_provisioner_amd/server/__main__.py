from .api_server import main

main()
