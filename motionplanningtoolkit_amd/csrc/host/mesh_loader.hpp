// mesh_loader.hpp -- triangle-soup reader replacing AssimpMeshLoader
// (utilities/assimp_mesh_loader.hpp:11-60) for the formats the reference ships:
// COLLADA (.dae), 3D Studio (.3ds) and Wavefront (.obj, the repo's fixture format).
//
// Semantics kept from the reference loader (Assimp 3.x, ReadFile(path, 0)):
//  * one submesh per Assimp aiMesh, in scene->mMeshes order: COLLADA <triangles>/<polylist>
//    elements in document order; 3DS faces split per material in material-list order;
//    OBJ `o`/`g` groups in file order;
//  * node transforms / <unit> / <up_axis> are ignored (the reference never reads them);
//  * faces that are not triangles are skipped (assimp_mesh_loader.hpp:50-53);
//  * coordinates are float32 (aiVector3D) widened to double (fcl::Vec3f).
// Number parsing is strtof (correctly rounded); Assimp's fast_atof may differ in the last
// float bit -- a documented convention, see DESIGN.md.
#pragma once
#include <string>
#include <vector>

namespace mpt_host {

struct SubMesh {
    std::string name;          // material / group name
    std::vector<double> tris;  // [n][9] vertex coordinates
    size_t size() const { return tris.size() / 9; }
};

struct MeshFile {
    std::vector<SubMesh> submeshes;
    bool error = false;
    std::string message;
    // all submeshes concatenated (StaticEnvironmentMeshHandler registers every one of them
    // with the same transform, utilities/meshhandler.hpp:38-50)
    std::vector<double> soup() const;
    // SimpleAgentMeshHandler keeps the LAST submesh with vertices and triangles
    // (utilities/meshhandler.hpp:124-134)
    std::vector<double> last_nonempty() const;
};

MeshFile load_mesh(const std::string &path);

}  // namespace mpt_host
