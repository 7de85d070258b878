# Generates the reference's ressources.h (normally produced by its CMakeLists.txt:10 configure_file)
# into oracle/_ref/gen/ -- a configure_file call of our own, not the reference's build system.  The asset root is
# ASSET_ROOT (the repo's assets/, laid out like the reference's models/ and textures/) when given, else REF.
# usage: cmake -DREF=/root/reference [-DASSET_ROOT=/root/repo/assets] -DOUT=oracle/_ref/gen/ressources.h -P gen_ressources.cmake
if(DEFINED ASSET_ROOT)
  set(RAYCASTER_ROOT_PATH ${ASSET_ROOT})
else()
  set(RAYCASTER_ROOT_PATH ${REF})
endif()
configure_file(${REF}/src/ressources.h.in ${OUT} @ONLY)
