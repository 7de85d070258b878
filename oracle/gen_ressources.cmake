# Generates the reference's ressources.h (normally produced by its CMakeLists.txt:10 configure_file)
# into oracle/_ref/gen/ — a configure_file call of our own, not the reference's build system.
# usage: cmake -DREF=/root/reference -DOUT=oracle/_ref/gen/ressources.h -P gen_ressources.cmake
set(RAYCASTER_ROOT_PATH ${REF})
configure_file(${REF}/src/ressources.h.in ${OUT} @ONLY)
